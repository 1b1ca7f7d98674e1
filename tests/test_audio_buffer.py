"""The streaming VAD chunker (src-tauri/src/audio.rs:29-241 AudioBuffer), through the C++ mirror in
nobs-whisper_amd/host/audio_buffer.cpp, against the numpy restatement in tests/oracle_py.py
(AudioBufferRef). CPU only: the buffer runs on the host.

Bar: bit-exact. Every dispatched chunk (samples and length), the overlap carry, last_speech_pos, the
noise floor and its frame count equal the restatement after every callback.
"""
import numpy as np
import pytest

from make_model import synthetic_pcm
from oracle_py import AudioBufferRef, rms_f32


@pytest.fixture(scope="module")
def wrs_host(wrs):
    return wrs


def test_audio_buffer_overlap(wrs_host):
    """audio.rs:806-831 test_audio_buffer_overlap, replayed."""
    sr = 16000
    buf = wrs_host.AudioBuffer.with_sample_rate(sr)
    i = np.arange(3 * sr, dtype=np.float32)
    speech = (np.sin(i * np.float32(0.01)) * np.float32(0.3)).astype(np.float32)
    buf.push_samples(speech)
    buf.push_samples(np.zeros(int(1.5 * sr), np.float32))
    assert buf.has_silence_boundary()
    assert buf.take_chunk_at_silence() is not None
    assert buf.overlap_len == sr * 200 // 1000


def test_calculate_rms_matches_sequential_f32(wrs_host):
    """audio.rs:586-595 test_calculate_rms values, and sequential f32 summation on random data."""
    assert wrs_host.calculate_rms(np.zeros(100, np.float32)) == 0.0
    assert abs(wrs_host.calculate_rms(np.ones(100, np.float32)) - 1.0) < 1e-6
    assert wrs_host.calculate_rms(np.zeros(0, np.float32)) == 0.0
    rng = np.random.default_rng(0)
    for n in (1, 7, 320, 960, 4099):
        x = (rng.standard_normal(n) * 0.1).astype(np.float32)
        assert np.float32(wrs_host.calculate_rms(x)) == rms_f32(x), n


def _state(b):
    return (len(b), b.last_speech_pos, b.overlap_len, b.noise_floor_frames, np.float32(b.get_noise_floor()))


def _ref_state(r):
    return (r._n, r.last_speech_pos, len(r.overlap), r.noise_floor_frames, np.float32(r.noise_floor))


def _recording(seed, sr, seconds):
    """speech-like stretches (synthetic_pcm), digital silences, low noise and one long continuous stretch
    (no silence: the forced split after 25 s)"""
    rng = np.random.default_rng(seed)
    parts, total = [], 0
    while total < seconds * sr:
        kind = rng.integers(0, 4)
        if kind == 0:
            x = synthetic_pcm(int(rng.integers(0, 50)), seconds=float(rng.uniform(1.0, 6.0)), sr=sr)
        elif kind == 1:
            x = np.zeros(int(rng.uniform(0.2, 1.6) * sr), np.float32)
        elif kind == 2:
            x = (rng.standard_normal(int(rng.uniform(0.3, 2.0) * sr)) * 0.002).astype(np.float32)
        else:
            t = np.arange(int(rng.uniform(0.5, 3.0) * sr), dtype=np.float32)
            x = (np.sin(t * np.float32(0.05)) * np.float32(0.2)).astype(np.float32)
        parts.append(x.astype(np.float32))
        total += len(x)
    return np.concatenate(parts)


@pytest.mark.parametrize("sr,seconds,block,seed", [(16000, 40, 160, 0), (16000, 35, 1024, 1), (8000, 60, 441, 2),
                                                   (48000, 12, 480, 3)])
def test_buffer_matches_restatement(wrs_host, sr, seconds, block, seed):
    """Random callback sizes over mixed recordings: chunks and state identical after every push."""
    rng = np.random.default_rng(100 + seed)
    x = _recording(seed, sr, seconds)
    if seed == 0:  # 27 s of uninterrupted tone: exceeds MAX_BUFFER_DURATION_S with no silence to split at
        t = np.arange(27 * sr, dtype=np.float32)
        x = np.concatenate([x, (np.sin(t * np.float32(0.03)) * np.float32(0.25)).astype(np.float32)])
    b, r = wrs_host.AudioBuffer(sr), AudioBufferRef(sr)
    pos, kinds = 0, []
    while pos < len(x):
        n = int(rng.integers(1, 2 * block))
        blk = x[pos:pos + n]
        pos += n
        b.push_samples(blk)
        r.push_samples(blk)
        assert b.has_silence_boundary() == r.has_silence_boundary()
        got, exp = b.take_chunk_at_silence(), r.take_chunk_at_silence()
        kind = 0
        if exp is None:
            got, exp = b.take_forced_chunk(), r.take_forced_chunk()
            kind = 1
        assert (got is None) == (exp is None), pos
        if exp is not None:
            kinds.append(kind)
            assert np.array_equal(got, exp), (pos, len(got), len(exp))
        assert _state(b) == _ref_state(r), pos
    assert kinds.count(0) >= 2, kinds
    if seed == 0:
        assert 1 in kinds, kinds
    rest_b, rest_r = b.take(), r.take()
    assert np.array_equal(rest_b, rest_r)
    assert _state(b) == _ref_state(r)


def test_unsupported_rate_is_an_error(wrs_host):
    with pytest.raises(ValueError):
        wrs_host.AudioBuffer(10)
