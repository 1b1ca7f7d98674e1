"""Audio front-end: the reference's silence chunking and 16 kHz resampler
(src-tauri/src/audio.rs) on the GPU (kernels/audio.hip through whisper_mi355x_find_silence_boundaries
/ whisper_mi355x_resample_chunk), against oracle/oracle_audio.cpp.

  * The reference's own tests (audio.rs:569-831) are replayed twice: on the oracle (CPU, pinning the
    restatement) and on the GPU mirror (whisper_rs.find_silence_boundaries / split_at_silences /
    resample_chunk), with the same signals and the same assertions.
  * Silence boundaries are integer outputs: GPU == oracle exactly, and every 20 ms window RMS is
    bit-identical (the thresholds are compared on those values), on single clips and ragged batches.
  * The resampler's values are "parity unpinned" beyond the restatement of rubato 0.15.0 (absent from
    the reference tree; its test pins only the length): GPU == the oracle's literal block-by-block
    pipeline (double precision) within RESAMPLE_TOL, lengths exact.
"""
import numpy as np
import pytest

import oracle_py as O

SR = 16000
# f32 dot products of 2*fsi (<= 2048) taps against a double-precision pipeline, |x| <= 1
RESAMPLE_TOL = 2e-5


def sine(n, step, amp):
    """(0..n).map(|i| (i as f32 * step).sin() * amp) in f32, as the reference's tests build signals."""
    i = np.arange(n, dtype=np.float32)
    return (np.sin(i * np.float32(step)).astype(np.float32) * np.float32(amp)).astype(np.float32)


def ref_signal(parts):
    """Concatenate (kind, seconds) parts as audio.rs's tests do: 'q' quiet 0.002 (x*0.1).sin(),
    'n' noise 0.005, 's' speech 0.3 (x*0.01).sin(), 'z' zeros."""
    out = []
    for kind, sec in parts:
        n = int(sec * SR)
        out.append({"q": lambda: sine(n, 0.1, 0.002), "n": lambda: sine(n, 0.1, 0.005),
                    "s": lambda: sine(n, 0.01, 0.3), "z": lambda: np.zeros(n, np.float32)}[kind]())
    return np.concatenate(out)


# audio.rs:619-662, 685-713, 715-744, 746-769, 771-802 (signal, expected boundary count)
REF_VAD_CASES = {
    "find_silence_in_audio": ([("q", 0.5), ("s", 2), ("z", 1), ("s", 2), ("z", 1), ("s", 2)], 2),
    "no_silence_returns_single_chunk": ([("q", 0.5), ("s", 10)], 0),
    "audio_with_silence_is_chunked": ([("q", 0.5), ("s", 2), ("z", 1), ("s", 2)], 1),
    "short_silence_not_split": ([("q", 0.5), ("s", 2), ("z", 0.5), ("s", 2)], 0),
    "adaptive_threshold_with_noisy_background": ([("n", 0.5), ("s", 2), ("n", 1), ("s", 2)], 1),
}


# ---- CPU: the oracle against the reference's own tests ---------------------------------------------
def test_oracle_calculate_rms():
    """audio.rs:585-594."""
    assert O.calculate_rms(np.zeros(100, np.float32)) < 0.001
    assert O.calculate_rms(np.full(100, 0.5, np.float32)) > 0.4


def test_oracle_estimate_noise_floor():
    """audio.rs:596-617."""
    a = ref_signal([("q", 0.5), ("s", 2)])
    assert O.estimate_noise_floor(a, SR) < 0.01


@pytest.mark.parametrize("name", list(REF_VAD_CASES))
def test_oracle_reference_vad_cases(name):
    parts, want = REF_VAD_CASES[name]
    a = ref_signal(parts)
    b = O.find_silence_boundaries(a, SR)
    assert len(b) == want, b
    chunks = O.split_at_silences(len(a), b, SR)
    assert len(chunks) == want + 1
    if not b:
        assert chunks == [(0, len(a))]


def test_oracle_split_with_overlap():
    """audio.rs:664-683: boundaries at 2 s and 4 s of 6 s -> 3 chunks, overlap 200 ms."""
    chunks = O.split_at_silences(6 * SR, [2 * SR, 4 * SR], SR)
    ov = SR * 200 // 1000
    assert [e - s for s, e in chunks] == [2 * SR, 2 * SR + ov, 2 * SR + ov]


def test_oracle_resample_ratio():
    """audio.rs:569-583: 48 kHz -> 16 kHz length within 10 % of n / 3."""
    x = sine(48000, 0.001, 1.0)
    y = O.resample(x, 48000)
    assert abs(len(y) - 16000) < 1600, len(y)


def test_mirror_split_matches_oracle():
    """whisper_rs.split_at_silences_with_overlap (pure indexing, the caller side) == the oracle."""
    from conftest import load_whisper_rs
    W = load_whisper_rs()
    a = np.arange(7 * SR, dtype=np.float32)
    for b in ([], [2 * SR], [2 * SR, 4 * SR], [SR // 10, 5 * SR], [0, 7 * SR, 8 * SR]):
        got = [(int(c[0]), int(c[-1]) + 1) for c in W.split_at_silences(a, b)]
        assert got == O.split_at_silences(len(a), b, SR), b


@pytest.mark.parametrize("rate", [48000, 44100, 22050, 8000])
def test_resample_operator_matches_oracle_pipeline(rate):
    """The product folds rubato's per-block FFT pipeline into one [2*fsi][fso] matrix (host code,
    no GPU needed to fetch it); applied in float64 it reproduces the oracle's literal 1024-sample
    call loop (saved frames, zero-padded last chunk, overlap-add, truncation)."""
    import ctypes as C
    from conftest import load_whisper_rs
    W = load_whisper_rs()
    L = W.lib()
    fsi, fso = C.c_int(), C.c_int()
    assert L.whisper_mi355x_resample_operator(rate, C.byref(fsi), C.byref(fso), None, 0) == 0
    fsi, fso = fsi.value, fso.value
    Wm = np.zeros((2 * fsi, fso), np.float32)
    assert L.whisper_mi355x_resample_operator(rate, None, None, Wm.ctypes.data_as(C.POINTER(C.c_float)), Wm.size) == 0
    rng = np.random.default_rng(rate)
    n = int(rate * 0.9) + 37
    x = (rng.standard_normal(n) * 0.2).astype(np.float32)
    ref = O.resample(x, rate)
    assert len(ref) == L.whisper_mi355x_resample_len(n, rate)
    nb = (len(ref) + fso - 1) // fso
    xp = np.concatenate([np.zeros(fsi), x.astype(np.float64), np.zeros((nb + 2) * fsi)])
    rows = np.stack([xp[m * fsi:(m + 2) * fsi] for m in range(nb)])
    y = (rows @ Wm.astype(np.float64)).reshape(-1)[:len(ref)]
    assert np.abs(y - ref).max() < 1e-5, np.abs(y - ref).max()


# ---- GPU ----------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", list(REF_VAD_CASES))
def test_gpu_reference_vad_cases(wrs, name):
    """audio.rs:619-802 through the GPU front-end; boundaries and chunk count as the reference asserts,
    and equal to the oracle's."""
    parts, want = REF_VAD_CASES[name]
    a = ref_signal(parts)
    b = wrs.find_silence_boundaries(a, SR)
    assert len(b) == want, b
    assert b == O.find_silence_boundaries(a, SR)
    chunks = wrs.split_at_silences(a, b)
    assert len(chunks) == (want + 1 if want else 1)
    if not want:
        assert len(chunks[0]) == len(a)


@pytest.mark.gpu
def test_gpu_estimate_noise_floor(wrs):
    """audio.rs:596-617 on the GPU's noise floor, equal to the oracle's bit for bit."""
    a = ref_signal([("q", 0.5), ("s", 2)])
    _, nf = wrs.find_silence_boundaries_batch([a], SR)
    assert nf[0] < 0.01
    assert np.float32(nf[0]) == np.float32(O.estimate_noise_floor(a, SR))


def speechlike(k, seconds, sr=SR):
    from make_model import synthetic_pcm
    x = synthetic_pcm(k, seconds=seconds, sr=sr)
    return x.astype(np.float32)


@pytest.mark.gpu
def test_gpu_window_rms_bit_exact_and_boundaries_ragged_batch(wrs):
    """A ragged batch (empty, shorter than one window, odd lengths, 30 s) in one call: every 20 ms
    window RMS bit-identical to the oracle's calculate_rms, boundaries and noise floors identical."""
    rng = np.random.default_rng(7)
    clips = [np.zeros(0, np.float32), speechlike(1, 0.013), speechlike(2, 30.0), speechlike(3, 12.345),
             (rng.standard_normal(SR * 3) * 0.01).astype(np.float32), speechlike(4, 25.2),
             np.concatenate([speechlike(5, 4.0), np.zeros(SR, np.float32), speechlike(6, 4.0)])]
    bounds, nfs, rms = wrs.find_silence_boundaries_batch(clips, SR, with_rms=True)
    ws = SR // 50
    for c, x in enumerate(clips):
        nw = len(x) // ws
        want = np.array([O.calculate_rms(x[w * ws:(w + 1) * ws]) for w in range(nw)], np.float32)
        assert len(rms[c]) == nw
        assert np.array_equal(rms[c].view(np.uint32), want.view(np.uint32)), c
        assert bounds[c] == O.find_silence_boundaries(x, SR), c
        assert np.float32(nfs[c]) == np.float32(O.estimate_noise_floor(x, SR)), c
    assert any(len(b) > 0 for b in bounds)


@pytest.mark.gpu
@pytest.mark.parametrize("sr", [16000, 48000])
def test_gpu_boundaries_many_clips(wrs, sr):
    """64 clips of 5-30 s in one launch == the oracle per clip (the app calls it at 16 kHz,
    state.rs:761; 48 kHz exercises 960-sample windows)."""
    rng = np.random.default_rng(sr)
    clips = [speechlike(10 + k, float(rng.uniform(5, 30)), sr=sr) for k in range(64)]
    bounds, _ = wrs.find_silence_boundaries_batch(clips, sr)
    for c, x in enumerate(clips):
        assert bounds[c] == O.find_silence_boundaries(x, sr), c


@pytest.mark.gpu
def test_gpu_resample_ratio(wrs):
    """audio.rs:569-583 through the GPU resampler."""
    x = sine(48000, 0.001, 1.0)
    y = wrs.resample_chunk(x, 48000)
    assert abs(len(y) - 16000) < 1600, len(y)


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [48000, 44100, 22050, 8000, 16000])
def test_gpu_resample_matches_oracle(wrs, rate):
    """Ragged batch (shorter than one FFT block, not a multiple of 1024, 30 s) against the oracle's
    literal rubato pipeline: lengths exact, values within RESAMPLE_TOL."""
    rng = np.random.default_rng(rate)
    lens = [0, 100, 1024, int(rate * 1.37) + 5, rate * 30]
    clips = [np.clip(speechlike(k, (n + 1) / rate, sr=rate)[:n] + (rng.standard_normal(n) * 0.05), -1, 1)
             .astype(np.float32) for k, n in enumerate(lens)]
    outs = wrs.resample_batch(clips, rate)
    for x, y in zip(clips, outs):
        ref = O.resample(x, rate) if len(x) < rate * 10 else None
        if ref is None:  # 30 s: compare a prefix (the oracle's direct DFTs are slow) and the length
            ref_head = O.resample(x[: rate * 3], rate)
            assert len(y) == wrs.lib().whisper_mi355x_resample_len(len(x), rate)
            k = len(ref_head) - 2048  # the tail of a truncated run differs (no later samples)
            assert np.abs(y[:k] - ref_head[:k]).max() < RESAMPLE_TOL
            continue
        assert len(y) == len(ref), (len(x), len(y), len(ref))
        if len(ref):
            assert np.abs(y - ref).max() < RESAMPLE_TOL, (len(x), np.abs(y - ref).max())
