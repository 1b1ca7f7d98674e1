"""The app's streaming recording path end to end (src-tauri/src/state.rs:113-168, 585-606, 655-798)
through the C++ StreamingSession (nobs-whisper_amd/host/audio_buffer.cpp): capture callbacks feed the
AudioBuffer VAD chunker on the host; every dispatched chunk is resampled 48 kHz -> 16 kHz on the GPU
(whisper_mi355x_resample_chunk) and transcribed by the WhisperEngine mirror on a worker thread, with the
previous non-empty text as context; stop() joins the worker, transcribes the remaining audio and joins
the texts.

Expected values are composed in Python from independently checked parts: the chunk sequence from the
numpy AudioBuffer restatement (tests/oracle_py.py, bit-exact on the CPU in test_audio_buffer.py), then
the same resample + transcribe calls in the app's order. This pins the orchestration (dispatch order,
context chaining, the remaining-audio rule, the join); the resampler and whisper_full are pinned to the
oracle by test_audio.py / test_gpu_parity.py.

The > 30 s remaining-audio branch (state.rs:757-778) cannot occur in streaming: the forced split keeps
the buffer under 25 s plus one callback.
"""
import numpy as np
import pytest

from make_model import synthetic_pcm
from oracle_py import AudioBufferRef, stream_callback_ref

pytestmark = pytest.mark.gpu

SR = 48000


def recording():
    z = lambda sec: np.zeros(int(sec * SR), np.float32)  # noqa: E731
    t = np.arange(27 * SR, dtype=np.float32)
    tone = (np.sin(t * np.float32(0.011)) * np.float32(0.2)).astype(np.float32) \
        * (0.6 + 0.4 * np.sin(t * np.float32(2e-4))).astype(np.float32)
    return np.concatenate([synthetic_pcm(3, 6.0, SR), z(1.0), synthetic_pcm(4, 4.0, SR), z(0.8),
                           tone, z(0.9), synthetic_pcm(5, 3.0, SR)]).astype(np.float32)


@pytest.mark.parametrize("language,vocab", [(None, True), ("en", False)])
def test_streaming_session_equals_app_order(wrs, language, vocab):
    from conftest import model_path
    x = recording()
    voc = wrs.DEFAULT_VOCABULARY if vocab else None
    eng = wrs.WhisperEngine()
    assert eng.load_model(model_path("tiny+conf")) == 0

    # the app's order, composed from the restated buffer and the same GPU calls
    ref = AudioBufferRef(SR)
    chunks = []
    for off in range(0, len(x), 480):  # 10 ms callbacks
        c = stream_callback_ref(ref, x[off:off + 480], 1)
        if c is not None:
            chunks.append(c)
    results, last = [], None
    for c in chunks:
        rc, text = eng.transcribe(wrs.resample_chunk(c, SR), language, voc, last)
        assert rc == 0
        if text:
            results.append(text)
            last = text
    rest = ref.take()
    if len(rest):
        pcm = wrs.resample_chunk(rest, SR)
        assert len(pcm) <= 30 * 16000
        if len(pcm) > 1600:
            rc, text = eng.transcribe(pcm, language, voc, results[-1] if results else None)
            assert rc == 0
            if text:
                results.append(text)
    final = " ".join(results).strip()
    assert len(chunks) >= 3

    s = wrs.StreamingSession(eng, SR, channels=1, language=language, vocabulary=voc)
    for off in range(0, len(x), 480):
        s.on_input(x[off:off + 480])
    got = s.stop()
    assert s.dispatched() == [len(c) for c in chunks]
    assert s.errors() == 0
    assert s.results() == results
    assert got == final
    s.close()
    print(f"streaming: {len(chunks)} chunks ({[round(len(c) / SR, 2) for c in chunks]} s), "
          f"{len(results)} texts, final {len(final)} chars")
