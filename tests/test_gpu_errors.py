"""Error returns instead of aborts, and the per-call state pattern of the reference.

whisper-rs maps a non-zero whisper_full return to WhisperError::TranscriptionError
(src-tauri/src/whisper.rs:127-129) and the streaming worker logs it and skips the chunk
(src-tauri/src/state.rs:157-159). The engine must therefore return, not abort, on a device error
(out of memory) or an unsupported input, and leave the context usable for the next chunk.

whisper.rs:83-85 creates a fresh state on every transcribe call and drops it at the end: the
context keeps released states (workspace + captured decode graphs) for the next whisper_init_state,
and a recycled state must behave exactly like a new one.
"""
import ctypes as C

import numpy as np
import pytest

from make_model import synthetic_pcm

pytestmark = pytest.mark.gpu

ERR_RUNTIME = -10  # include/whisper_mi355x.h WHISPER_MI355X_ERR_RUNTIME


def seg_ints(segs):
    return [([t[0] for t in s.tokens], s.t0, s.t1, s.text) for s in segs]


def test_out_of_memory_batch_returns_error_and_context_survives(wrs):
    """A batch whose workspace cannot fit in HBM (120000 clips of large-v3-2L: the self-KV cache alone
    needs 550 GB) fails with WHISPER_MI355X_ERR_RUNTIME; the same state and context then transcribe a
    clip exactly as a fresh context does."""
    from conftest import model_path
    path = model_path("large-v3-2L+conf")
    pcm = synthetic_pcm(0)
    p = wrs.reference_full_params("en")
    ref_ctx = wrs.WhisperContext(path, dtype=wrs.BF16)
    st = ref_ctx.create_state()
    assert st.full(p, pcm) == 0
    ref = seg_ints(st.segments())
    st.close()
    ref_ctx.close()
    assert ref

    ctx = wrs.WhisperContext(path, dtype=wrs.BF16)
    st = ctx.create_state()
    tiny = np.zeros(1600, np.float32)
    rc = st.full_batch(p, [tiny] * 120000)
    assert rc == ERR_RUNTIME, rc
    assert st.full_n_segments() == 0
    assert st.info()["cap_jobs"] == 0  # the half-built workspace was released as a whole
    assert st.full(p, pcm) == 0         # same state, same context
    assert seg_ints(st.segments()) == ref
    st.close()
    st = ctx.create_state()             # and a new state on the same context
    assert st.full(p, pcm) == 0
    assert seg_ints(st.segments()) == ref
    st.close()
    ctx.close()


def test_unsupported_sample_rate_returns_error(wrs):
    """audio.rs-style silence search at a sample rate whose 20 ms window does not fit the kernel's LDS
    staging (4 MHz: 80000-sample windows): -1, not an abort; a supported rate works afterwards."""
    L = wrs.lib()
    x = synthetic_pcm(0, seconds=10.0)  # 160000 samples: two 20 ms windows at 4 MHz
    ptrs = (C.c_void_p * 1)(x.ctypes.data)
    n = (C.c_int * 1)(len(x))
    counts = (C.c_int * 1)()
    bnd = (C.c_int * 8)()
    ip = C.POINTER(C.c_int)
    rc = L.whisper_mi355x_find_silence_boundaries(0, ptrs, n, 1, 4_000_000, False, C.cast(counts, ip),
                                                  C.cast(bnd, ip), 8, None, None, 0)
    assert rc == -1, rc
    rc = L.whisper_mi355x_find_silence_boundaries(0, ptrs, n, 1, 16000, False, C.cast(counts, ip),
                                                  C.cast(bnd, ip), 8, None, None, 0)
    assert rc == 0, rc


def test_encode_without_mel_is_an_error(wrs, tiny_model):
    """whisper_encode on a state that never computed a mel returns an error, also when the state was
    recycled from the pool (its workspace still holds the previous owner's mel)."""
    L = wrs.lib()
    ctx = wrs.WhisperContext(tiny_model, dtype=wrs.F16)
    st = ctx.create_state()
    pcm = synthetic_pcm(1)
    assert st.full(wrs.reference_full_params("en"), pcm) == 0
    st.close()
    st = ctx.create_state()
    assert st.info()["pooled"]
    assert L.whisper_encode_with_state(ctx.ptr, st.ptr, 0, 1) != 0
    st.close()
    ctx.close()


@pytest.mark.parametrize("shape,dtype", [("tiny+conf", "F16"), ("large-v3-2L+conf", "BF16")])
def test_recycled_state_equals_fresh_state(wrs, monkeypatch, shape, dtype):
    """The app's pattern (whisper.rs:83-85): state per call. Calls 2..4 reuse the pooled workspace and
    its decode graphs (no allocation, no capture) and must give the same results as a fresh context,
    including the prompt carry-over that a recycled state must NOT inherit (prompt_past, rng)."""
    from conftest import model_path
    path = model_path(shape)
    p = wrs.reference_full_params("en", initial_prompt=wrs.DEFAULT_VOCABULARY)
    clips = [synthetic_pcm(k, seconds=25.0) for k in range(3)]
    dt = getattr(wrs, dtype)

    def fresh(pcm):
        monkeypatch.setenv("WHISPER_MI355X_STATE_POOL", "0")
        c = wrs.WhisperContext(path, dtype=dt)
        s = c.create_state()
        assert not s.info()["pooled"]
        assert s.full(p, pcm) == 0
        r = seg_ints(s.segments())
        s.close()
        c.close()
        monkeypatch.delenv("WHISPER_MI355X_STATE_POOL")
        return r

    refs = [fresh(x) for x in clips]
    ctx = wrs.WhisperContext(path, dtype=dt)
    for i, x in enumerate(clips + clips[:1]):
        st = ctx.create_state()
        assert st.info()["pooled"] == (i > 0)
        assert st.full(p, x) == 0
        assert seg_ints(st.segments()) == refs[i % 3], i
        if i > 0:
            assert st.info()["graphs"] >= 1
        st.close()
    ctx.close()


def test_state_outliving_its_context(wrs):
    """A garbage collector may finalise a context before its states (the round-3 suite crashed at
    interpreter exit that way): whisper_free orphans the states a caller still holds, and a later
    whisper_free_state releases them without touching the freed context. The Python wrapper also
    closes a context's states first."""
    from conftest import model_path
    path = model_path("tiny.en")
    ctx = wrs.WhisperContext(path)
    L = ctx.L
    a, b = ctx.create_state(), ctx.create_state()
    assert a.full(wrs.reference_full_params("en"), synthetic_pcm(0)) == 0
    b.close()  # pooled: whisper_free destroys it with the pool
    raw = a.ptr
    a.ptr = None  # the wrapper no longer owns it: free it by hand after the context
    L.whisper_free(ctx.ptr)
    ctx.ptr = None
    L.whisper_free_state(raw)  # orphan: must not touch the freed context
    # wrapper order: closing the context closes its live states first
    ctx2 = wrs.WhisperContext(path)
    st = ctx2.create_state()
    ctx2.close()
    assert st.ptr is None


def test_cross_cache_regrow_drops_stale_graphs(wrs, monkeypatch):
    """one state runs a direct-form batch of 40 clips (workspace for 64 slots, no cross
    K/V cache), then cache-form batches of 8 clips (decode graphs captured for <= 8 active clips over
    the cache) and 16 clips (the cache is reallocated larger). The 8-clip batch run again after the
    reallocation replays graphs for <= 8 clips: they must have been dropped with the old cache, so every
    result equals a fresh state's, bit for bit."""
    from conftest import model_path
    path = model_path("tiny+conf")
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    clips = [synthetic_pcm(k % 12, seconds=30.0 - k % 5) for k in range(40)]

    def run(st, cl):
        assert st.full_batch(p, cl) == 0
        return [seg_ints(st.batch_segments(j)) for j in range(len(cl))]

    monkeypatch.setenv("WHISPER_MI355X_STATE_POOL", "0")  # every state starts with no workspace
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    fresh = {}
    for key, cl in (("a", clips[:8]), ("b", clips[8:24])):
        s = ctx.create_state()
        fresh[key] = run(s, cl)
        s.close()
    st = ctx.create_state()
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "direct")
    run(st, clips)
    assert st.info()["direct"]
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    assert run(st, clips[:8]) == fresh["a"]
    assert not st.info()["direct"]
    assert run(st, clips[8:24]) == fresh["b"]
    assert run(st, clips[:8]) == fresh["a"]
    st.close()
    ctx.close()
