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
