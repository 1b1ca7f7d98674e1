"""Pipelined greedy decoding (engine.cpp decode_pipelined): the next decode step is launched before the host
has processed the last one, every row's token / position / logits-rule state advanced on the device
(kernels/logits.hip decode_advance_kernel). Results must be the per-step path's bits (WHISPER_MI355X_PIPE=0):
token ids, timestamps, text and per-window decisions of whisper_full (the reference's FullParams, greedy
attempt, whisper.rs:88-124), one clip through the persistent step and batches through the launch chain in both
cross forms, real termination (EOT / timestamps end each window: the speculative step at an attempt's end) and
fixed work."""
import numpy as np
import pytest

from make_model import synthetic_pcm

pytestmark = pytest.mark.gpu


def _run(wrs, path, clips, pipe, monkeypatch, cross=None, fixed=0, pipe_min=None):
    monkeypatch.setenv("WHISPER_MI355X_PIPE", "1" if pipe else "0")
    if pipe_min is not None:
        monkeypatch.setenv("WHISPER_MI355X_PIPE_MIN", str(pipe_min))
    if cross:
        monkeypatch.setenv("WHISPER_MI355X_CROSS", cross)
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    st = ctx.create_state()
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    assert st.full_batch(p, clips, fixed_tokens=fixed) == 0
    out = []
    for k in range(len(clips)):
        segs = st.batch_segments(k)
        out.append(([([t[0] for t in s.tokens], s.t0, s.t1, s.text) for s in segs], st.decisions(k)))
    assert st.pdec_give_ups() == 0
    st.close()
    ctx.close()
    return out


# (pipe_min 2: pipelining from the third token of every attempt, so that short windows end inside a pipelined
# run and the speculative step at an attempt's end is exercised; fixed work: 64 tokens with EOT suppressed)
@pytest.mark.parametrize("shape,n,cross,fixed,pipe_min", [
    ("base+conf", 1, None, 0, 2), ("base+conf", 1, None, 64, None), ("tiny+conf", 3, None, 0, 2),
    ("small-4L+conf", 40, "direct", 0, 2), ("small-4L+conf", 40, "direct", 48, None), ("small-4L+conf", 8, "cache", 0, 2)])
def test_pipelined_equals_per_step(wrs, monkeypatch, shape, n, cross, fixed, pipe_min):
    from conftest import model_path
    path = model_path(shape)
    clips = [synthetic_pcm(k, seconds=30.0 if k % 2 == 0 else 21.0) for k in range(n)]
    a = _run(wrs, path, clips, True, monkeypatch, cross=cross, fixed=fixed, pipe_min=pipe_min)
    b = _run(wrs, path, clips, False, monkeypatch, cross=cross, fixed=fixed, pipe_min=pipe_min)
    ntok = sum(len(t) for segs, _ in a for t, *_ in segs)
    print(f"{shape} x {n} fixed {fixed}: {ntok} tokens")
    assert ntok > 0
    assert a == b


def test_pipelined_abort_callback(wrs, monkeypatch):
    """whisper_full's abort callback (asked before every decode step, whisper.rs passes none but the ABI has
    it) with pipelined decoding: the call returns 0 with the windows finished before the abort, a prefix of an
    unaborted run's segments, as on the per-step path; the state then transcribes the clip again (with the
    aborted call's text as its prompt_past, so not the fresh result)."""
    import ctypes as C
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_PIPE_MIN", "2")
    cbt = C.CFUNCTYPE(C.c_bool, C.c_void_p)
    pcm = synthetic_pcm(5, seconds=75.0)

    def run(pipe, limit):
        monkeypatch.setenv("WHISPER_MI355X_PIPE", "1" if pipe else "0")
        ctx = wrs.WhisperContext(model_path("base+conf"), dtype=wrs.F16)
        st = ctx.create_state()
        calls = [0]

        def cb(_):
            calls[0] += 1
            return limit is not None and calls[0] >= limit
        f = cbt(cb)
        p = wrs.reference_full_params("en")
        p.temperature_inc = 0.0
        p.abort_callback = C.cast(f, C.c_void_p)
        assert st.full(p, pcm) == 0
        segs = [([t[0] for t in s.tokens], s.t0, s.t1, s.text)
                for s in (st.get_segment(i) for i in range(st.full_n_segments()))]
        p.abort_callback = None
        assert st.full(p, pcm) == 0  # the same state, no abort: the unaborted result
        again = [([t[0] for t in s.tokens], s.t0, s.t1, s.text)
                 for s in (st.get_segment(i) for i in range(st.full_n_segments()))]
        st.close()
        ctx.close()
        return segs, again, calls[0]

    full, _, n_calls = run(True, None)
    assert len(full) >= 2 and n_calls > 20
    for pipe in (True, False):
        segs, again, _ = run(pipe, n_calls // 2)
        assert len(segs) < len(full) and segs == full[:len(segs)], (pipe, len(segs), len(full))
        assert len(again) > 0
    print(f"{len(full)} segments, {n_calls} callback calls unaborted")


def test_pipelined_row_at_context_end_beside_continuing_row(wrs, monkeypatch):
    """the speculative step k + 1 runs for every row, so a row at its 220-token limit with a
    full prompt (multilingual, no_timestamps: 1 + 224 + 4 = 229 tokens) would have been decoded at position
    229 + 219 = 448, one past the self cache and the positional table, while another row still decoded. Here
    clip 5 (60 s) ends its first window at step 156 (EOT: tiny+conf+eot, make_model.CONF_EOT_BOOST) and starts
    its second while clip 1 runs its first window to the limit: the pipelined run must equal the per-step one."""
    from conftest import model_path
    path = model_path("tiny+conf+eot")
    clips = [synthetic_pcm(5, seconds=60.0), synthetic_pcm(1, seconds=60.0)]
    prompt = " ".join(f"word{k} alpha beta" for k in range(120))  # ~970 tokens: prompt_past keeps the last 224

    def run(pipe):
        monkeypatch.setenv("WHISPER_MI355X_PIPE", "1" if pipe else "0")
        monkeypatch.setenv("WHISPER_MI355X_PIPE_MIN", "2")
        ctx = wrs.WhisperContext(path, dtype=wrs.F16)
        st = ctx.create_state()
        p = wrs.reference_full_params("en")
        p.temperature_inc = 0.0
        p.no_timestamps = True
        p.initial_prompt = prompt.encode()
        assert st.full_batch(p, clips) == 0
        out = [([([t[0] for t in s.tokens], s.t0, s.t1, s.text) for s in st.batch_segments(k)], st.decisions(k))
               for k in range(len(clips))]
        assert st.pdec_give_ups() == 0
        st.close()
        ctx.close()
        return out

    a, b = run(True), run(False)
    # the scenario: clip 5's first window ended early (EOT), clip 1's ran to the limit (no result: failed)
    d5, d1 = b[0][1], b[1][1]
    print("decisions clip 5:", [(d["seek"], d["result_len0"], d["failed0"]) for d in d5],
          "clip 1:", [(d["seek"], d["result_len0"], d["failed0"]) for d in d1])
    assert len(d5) == 2 and 0 < d5[0]["result_len0"] < 200, d5
    assert d1[0]["failed0"] == 1 and d1[0]["result_len0"] == 0, d1
    assert a == b


def test_pipelined_active_rows_cross_64(wrs, monkeypatch):
    """when an attempt ends inside a pipelined run, the speculative step's results stand for
    the rows still decoding only if a step of that many rows computes the same bits (step_variant). 70 clips of
    staggered lengths in the cache form (tiny+conf: windows end on timestamps at clip-dependent steps) take the
    active count across 64, where the logits GEMM changes kernel; results must equal the per-step path's."""
    from conftest import model_path
    path = model_path("tiny+conf")
    clips = [synthetic_pcm(k % 24, seconds=10.0 + 0.5 * (k % 37)) for k in range(70)]
    a = _run(wrs, path, clips, True, monkeypatch, cross="cache", pipe_min=2)
    b = _run(wrs, path, clips, False, monkeypatch, cross="cache", pipe_min=2)
    assert a == b
