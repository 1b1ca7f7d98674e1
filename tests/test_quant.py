"""GGML quantized model files (whisper.cpp's q4_0 / q4_1 / q5_0 / q5_1 / q8_0, the
formats `whisper-quantize` writes and the reference's model download list ships as *-q5_*.bin).

The oracle's loader is checked block by block against an independent numpy restatement of ggml's
dequantize_row_* (tools/make_model.py dequantize_rows): exact f32 dequantization in mode 0; in mode 1
(ggml numerics) the matmul operands are those values rounded to f16 (ggml's GPU back-ends
dequantize blocks into half tiles) while the decoder's token lookup keeps the exact f32 rows
(ggml_get_rows dequantizes to f32). The GPU tests then require the engine's whisper_full on the
quantized files to equal the oracle's token for token. Parity of the quantizer itself is unpinned
(ggml is not in the reference tree); the files are self-consistent: what is written is what is read.
"""
import numpy as np
import pytest

from make_model import GGML_TYPES, QUANT_SKIP, read_tensors
from oracle_py import Oracle

QTYPES = list(GGML_TYPES)


@pytest.mark.parametrize("qtype", QTYPES)
def test_oracle_dequant_matches_numpy(qtype):
    from conftest import model_path
    from make_model import dequantize_rows
    path = model_path("micro+" + qtype)
    raw = read_tensors(path)
    quantized = {n for n, (tt, ne, _) in raw.items() if tt == GGML_TYPES[qtype]}
    # every 2-D tensor except whisper.cpp's skip list
    assert quantized == {n for n, (tt, ne, _) in raw.items() if len(ne) == 2 and n not in QUANT_SKIP}
    assert "decoder.token_embedding.weight" in quantized and "encoder.blocks.0.mlp.0.weight" in quantized
    o0, o1 = Oracle(path, mode=0, n_threads=2), Oracle(path, mode=1, n_threads=2)
    try:
        for name in sorted(quantized):
            tt, ne, b = raw[name]
            want = dequantize_rows(b, qtype, int(np.prod(ne)))
            np.testing.assert_array_equal(o0.tensor(name), want, err_msg=name)
            np.testing.assert_array_equal(o1.tensor(name), want.astype(np.float16).astype(np.float32), err_msg=name)
        te = dequantize_rows(raw["decoder.token_embedding.weight"][2], qtype, o0.n_vocab * o0.d)
        np.testing.assert_array_equal(o1.tensor("decoder.token_embedding.weight", lookup=True), te)
    finally:
        o0.close()
        o1.close()


def test_quant_header_ftype():
    """ftype = GGML_FTYPE_MOSTLY_Q5_0 (8) + 1000 * GGML_QNT_VERSION (2)."""
    import struct
    from conftest import model_path
    with open(model_path("micro+q5_0"), "rb") as f:
        f.read(4)
        assert struct.unpack("<11i", f.read(44))[10] == 2008


def test_quant_oracle_full_runs():
    from conftest import model_path
    from make_model import synthetic_pcm
    from oracle_py import reference_params
    o = Oracle(model_path("tiny+conf+q5_0"), mode=1, n_threads=8)
    try:
        res = o.full(synthetic_pcm(0, seconds=11.0), reference_params("en"))
        assert res["rc"] == 0 and len(res["segments"]) > 0
    finally:
        o.close()


# ---- GPU: whisper_full on quantized files, f16, exact against the oracle ------------------------------
# f16 engine logits stay within ~0.015 of the oracle's (tools/debug/tf_logits.py): a step whose
# oracle margin (top-2 log-probability gap, or the timestamp rule's gap) is below F16_GAP could
# legitimately flip, so the exact comparison is only made on clips without one
F16_GAP = 0.05
QUANT_CASES = [
    # shape, clip seed; every oracle window decided at t = 0 with the reference's FullParams, and no
    # greedy step a close call (both asserted)
    ("tiny+conf+q5_0", 1), ("tiny.en+conf+q4_0", 0), ("base+conf+q8_0", 2), ("small-4L+conf+q5_1", 1),
    ("large-v3-2L+conf+q5_0", 0), ("large-v3-turbo-2L+conf+q4_1", 1),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cross", ["direct", "cache"])
@pytest.mark.parametrize("shape,clip", QUANT_CASES)
def test_quant_full_f16_exact(wrs, monkeypatch, cross, shape, clip):
    from conftest import model_path
    from make_model import synthetic_pcm
    from oracle_py import reference_params
    from test_gpu_configs import assert_decisions_match, gpu_full, ref_ints, seg_ints
    pcm = synthetic_pcm(clip)
    o = Oracle(model_path(shape), mode=1, n_threads=16)
    ref = o.full(pcm, reference_params("en"))
    o.close()
    assert all(d["temp_idx"] == 0 for d in ref["decisions"]), ref["decisions"]
    assert min(ref["margins"]) > F16_GAP, sorted(ref["margins"])[:3]
    segs, dec, _ = gpu_full(wrs, model_path(shape), wrs.F16, pcm, "en", cross=cross, monkeypatch=monkeypatch)
    assert_decisions_match(dec, ref)
    assert seg_ints(segs) == ref_ints(ref)
    assert [s.text for s in segs] == [s["text"] for s in ref["segments"]]


# ---- GPU: the blocks stay quantized in HBM ----------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("qtype", QTYPES)
def test_quant_arena_keeps_blocks(wrs, qtype):
    """A quantized file's projection matrices stay as GGML blocks in the device arena (q5_0: 0.69
    bytes per weight instead of 2): the arena is smaller than WHISPER_MI355X_QUANT_EXPAND=1's (the
    round-2 dequantize-at-load layout) by exactly the projections' expansion."""
    import ctypes as C
    import os
    from conftest import model_path
    L = wrs.lib()

    def arena(path, expand=False):
        if expand:
            os.environ["WHISPER_MI355X_QUANT_EXPAND"] = "1"
        try:
            ctx = wrs.WhisperContext(path, dtype=wrs.F16)
        finally:
            os.environ.pop("WHISPER_MI355X_QUANT_EXPAND", None)
        p, n = C.c_void_p(), C.c_size_t()
        assert L.whisper_mi355x_weight_arena(ctx.ptr, C.byref(p), C.byref(n)) == 0
        ctx.close()
        return n.value

    f16 = arena(model_path("large-v3-2L+conf"))
    q = arena(model_path("large-v3-2L+conf+" + qtype))
    qx = arena(model_path("large-v3-2L+conf+" + qtype), expand=True)
    bpw = {"q4_0": 18 / 32, "q4_1": 20 / 32, "q5_0": 22 / 32, "q5_1": 24 / 32, "q8_0": 34 / 32}[qtype]
    d = 1280
    proj = (2 * 12 + 2 * 14) * d * d  # 2 encoder (QKV, out, FC1, FC2) + 2 decoder layers (+ cross Q, out)
    # the expanded layout = the f16 file's + the exact f32 embedding rows a quantized file keeps for
    # the token lookup (ggml_get_rows dequantizes to f32): V x d x 4 bytes
    assert qx == f16 + 51866 * d * 4 or abs(qx - f16 - 51866 * d * 4) < 4096, (qx, f16)
    assert abs((qx - q) - proj * (2 - bpw)) < 0.01 * proj, (qx, q, proj)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["tiny+conf+q5_0", "small-4L+conf+q5_1"])
def test_quant_batch_equals_single(wrs, monkeypatch, shape):
    """40 clips with the small-M path forced for every decode step (its GEMMs read the blocks in
    32-row chunks) == whisper_full_with_state per clip, bit for bit (cache form): a row's sums do not
    depend on the rows beside it on this path."""
    from conftest import model_path
    from make_model import synthetic_pcm
    from test_gpu_configs import seg_ints
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    monkeypatch.setenv("WHISPER_MI355X_QSMALL_MAX", "64")
    monkeypatch.setenv("WHISPER_MI355X_PDEC", "0")  # singles on the small-M path too
    monkeypatch.setenv("WHISPER_MI355X_XWIDE_MAX", "0")  # the 256-thread cross step at every clip count
    ctx = wrs.WhisperContext(model_path(shape), dtype=wrs.F16)
    clips = [synthetic_pcm(k % 12, seconds=30.0 - k % 5) for k in range(40)]
    p = wrs.reference_full_params("en")
    st = ctx.create_state()
    assert st.full_batch(p, clips) == 0
    batch = [seg_ints(st.batch_segments(j)) for j in range(40)]
    st.close()
    for j in (0, 31, 32, 39):
        st = ctx.create_state()
        assert st.full(p, clips[j]) == 0
        assert seg_ints(st.segments()) == batch[j], j
        st.close()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cross", ["direct", "cache"])
@pytest.mark.parametrize("shape,clip", [("tiny+conf+q5_0", 1), ("large-v3-2L+conf+q5_0", 0)])
def test_quant_batch_dequant_path_exact(wrs, monkeypatch, cross, shape, clip):
    """Decode steps of more than 32 clips of a quantized file dequantize each layer's blocks once per
    step (one launch) and run the split-K GEMMs: 40 clips, the oracle's exact case at rows 0, 33 and 39,
    each equal to the oracle (f16, exact; the same bar as test_quant_full_f16_exact)."""
    from conftest import model_path
    from make_model import synthetic_pcm
    from oracle_py import reference_params
    from test_gpu_configs import ref_ints, seg_ints
    pcm = synthetic_pcm(clip)
    o = Oracle(model_path(shape), mode=1, n_threads=16)
    ref = o.full(pcm, reference_params("en"))
    o.close()
    assert min(ref["margins"]) > F16_GAP
    monkeypatch.setenv("WHISPER_MI355X_CROSS", cross)
    ctx = wrs.WhisperContext(model_path(shape), dtype=wrs.F16)
    rows = (0, 33, 39)
    clips = [pcm if j in rows else synthetic_pcm(j % 12 + 2, seconds=30.0 - j % 5) for j in range(40)]
    st = ctx.create_state()
    assert st.full_batch(wrs.reference_full_params("en"), clips) == 0
    for j in rows:
        segs = st.batch_segments(j)
        assert seg_ints(segs) == ref_ints(ref), j
        assert [s.text for s in segs] == [s["text"] for s in ref["segments"]], j
    st.close()
    ctx.close()
