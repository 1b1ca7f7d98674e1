"""The app's streaming transcription replayed end to end (the context carry-over between chunks
must stay exercised after the round-4 removal of the threaded StreamingSession restatement).

What runs, in the reference's order, on one thread (the reference's threads only hand data along):
  * recording callback (src-tauri/src/state.rs:586-606): every 20 ms block goes into AudioBuffer
    (audio.rs:60-86 push_samples); a chunk is dispatched by take_chunk_at_silence (audio.rs:111-158),
    else take_forced_chunk (audio.rs:161-225);
  * transcription worker (state.rs:113-168): resample_chunk (audio.rs:331-337) then
    WhisperEngine::transcribe(chunk, language, vocabulary, last_context); a non-empty result becomes
    last_context and is collected;
  * stop path (state.rs:655-798): the buffer's remaining audio (audio.rs:299-327 stop_recording: take);
    above 0.1 s it is transcribed with the last collected result as context, split at silence
    boundaries first when it exceeds 30 s (audio.rs:400-507); all results joined with " " and trimmed.
The product side is the C++ AudioBuffer mirror, the GPU VAD / resampler entry points and the C++
WhisperEngine mirror over the HIP engine. The expected side is the same control flow over the test
infrastructure: oracle_py.AudioBufferRef (numpy restatement of audio.rs), the oracle's silence
boundaries, and the CPU oracle's whisper_full behind whisper.rs:131-144's text assembly
(tests/test_gpu_mirror.py expected_text). The recording is at 16 kHz, where resample_chunk is the
identity (audio.rs:332-334), so the comparison is exact; the 48 kHz resampler has its own tests
(tests/test_audio.py).
"""
import numpy as np
import pytest

from make_model import synthetic_pcm
from oracle_py import AudioBufferRef, Oracle, find_silence_boundaries, split_at_silences
from test_gpu_mirror import expected_text

pytestmark = pytest.mark.gpu

# tiny+conf: every chunk's window is decided at t = 0 (no sampled fallback) and no greedy step of the
# oracle is closer than 0.11 nats (the f16 near-tie rule's 0.05), so the comparison is exact; base+conf
# falls back on one short chunk with the reference's logprob threshold
SHAPE = "tiny+conf"
SR = 16000


def recording():
    """~70 s: five synthetic utterances (0.7-1 s internal pauses) separated by 1.2 s of low noise: the
    buffer dispatches 17 chunks of 1.7-8 s at silences and leaves 0.85 s for the stop path."""
    rng = np.random.default_rng(7)
    parts = []
    for k, sec in enumerate((9.0, 27.0, 6.0, 14.0, 8.5)):
        parts.append(synthetic_pcm(20 + k, seconds=sec))
        parts.append((rng.standard_normal(int(1.2 * SR)) * 0.002).astype(np.float32))
    return np.concatenate(parts).astype(np.float32)


def record(buf, rec):
    chunks = []
    for off in range(0, len(rec), SR // 50):
        buf.push_samples(rec[off:off + SR // 50])
        c = buf.take_chunk_at_silence()
        if c is None:
            c = buf.take_forced_chunk()
        if c is not None:
            chunks.append(np.asarray(c, np.float32))
    return chunks, np.asarray(buf.take(), np.float32)


def replay(chunks, remaining, transcribe, boundaries):
    results, last = [], None
    for c in chunks:  # the worker
        text = transcribe(c, last)
        if text:
            last = text
            results.append(text)
    if len(remaining) > 1600:  # the stop path
        pieces = [remaining]
        if len(remaining) > 30 * SR:
            pieces = [remaining[a:b] for a, b in split_at_silences(len(remaining), boundaries(remaining), SR)]
        for p in pieces:
            text = transcribe(p, results[-1] if results else None)
            if text:
                results.append(text)
    return " ".join(results).strip(), results


def test_streaming_worker_and_stop_replay(wrs):
    from conftest import model_path
    path = model_path(SHAPE)
    rec = recording()
    got_chunks, got_rest = record(wrs.AudioBuffer.with_sample_rate(SR), rec)
    exp_chunks, exp_rest = record(AudioBufferRef(SR), rec)
    assert len(got_chunks) == len(exp_chunks) >= 3, (len(got_chunks), len(exp_chunks))
    for a, b in zip(got_chunks, exp_chunks):
        assert np.array_equal(a, b)
    assert np.array_equal(got_rest, exp_rest)

    eng = wrs.WhisperEngine()
    assert eng.load_model(path) == 0

    def gpu_transcribe(pcm, ctx):
        x = wrs.resample_chunk(pcm, SR)  # audio.rs:331-337: the identity at 16 kHz
        assert np.array_equal(np.asarray(x, np.float32), pcm)
        rc, text = eng.transcribe(x, "en", wrs.DEFAULT_VOCABULARY, ctx)
        assert rc == 0
        return text

    o = Oracle(path, mode=1, n_threads=16)

    def oracle_transcribe(pcm, ctx):
        return expected_text(wrs, o, pcm, "en", wrs.build_initial_prompt(wrs.DEFAULT_VOCABULARY, ctx))

    got, got_parts = replay(got_chunks, got_rest, gpu_transcribe, lambda a: wrs.find_silence_boundaries(a, SR))
    exp, exp_parts = replay(exp_chunks, exp_rest, oracle_transcribe, lambda a: find_silence_boundaries(a, SR))
    o.close()
    assert len(exp_parts) >= 3  # several chunks carried a previous result as context
    assert got_parts == exp_parts
    assert got == exp
    print(f"streaming replay: {len(got_chunks)} chunks + {len(got_rest) / SR:.1f} s at stop, "
          f"{len(got_parts)} results, {len(got)} chars identical")
