"""Kernel-level GPU parity: the MFMA GEMM (both staging variants, split-K path) against a float64
numpy reference of the same f16 operands. Tolerance: |err| <= 1e-4 * sum_k |a_k b_k| + 1e-5 (f32
accumulation of f16-exact products; order differs from numpy)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(wrs, micro_model):
    c = wrs.WhisperContext(micro_model, dtype=wrs.F16)
    yield c
    c.close()


def _dev(wrs, ctx, arr):
    L = wrs.lib()
    p = L.whisper_mi355x_dev_alloc(ctx.ptr, arr.nbytes)
    assert p
    L.whisper_mi355x_memcpy(ctx.ptr, C.c_void_p(p), arr.ctypes.data, arr.nbytes, 1)
    return p


def _run_gemm(wrs, ctx, A, B, bias, variant, reps=1, epi=4):
    L = wrs.lib()
    L.whisper_mi355x_debug_gemm.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                            C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_float)]
    L.whisper_mi355x_set_gemm_variant.argtypes = [C.c_int]
    M, K = A.shape
    N = B.shape[0]
    pa, pb, pbias = _dev(wrs, ctx, A), _dev(wrs, ctx, B), _dev(wrs, ctx, bias)
    out = np.zeros((M, N), np.float32 if epi in (2, 4) else np.float16)
    po = _dev(wrs, ctx, out)
    L.whisper_mi355x_set_gemm_variant(variant)
    ms = C.c_float()
    assert L.whisper_mi355x_debug_gemm(ctx.ptr, epi, C.c_void_p(pa), M, K, C.c_void_p(pb), N, C.c_void_p(pbias),
                                       C.c_void_p(po), reps, C.byref(ms)) == 0
    L.whisper_mi355x_set_gemm_variant(-1)
    L.whisper_mi355x_memcpy(ctx.ptr, out.ctypes.data, C.c_void_p(po), out.nbytes, 2)
    for p in (pa, pb, pbias, po):
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
    return out, ms.value


@pytest.mark.parametrize("M,N,K", [(1500 * 2 + 5, 1280, 1280), (3000, 51866, 384), (257, 384, 1536), (2048, 512, 64),
                                   (1500, 1024, 128), (4096, 1280, 5120),
                                   (32, 1280, 5120), (128, 3840, 1280), (7, 51866, 384),
                                   (100, 1280, 5120), (128, 5120, 1280), (1, 448, 384)])
@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3])
def test_gemm_matches_numpy(wrs, ctx, M, N, K, variant):
    rng = np.random.default_rng(M * 7 + N + K)
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    out, _ = _run_gemm(wrs, ctx, A, B, bias, variant)
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    ref = A64 @ B64.T + bias
    bound = 1e-4 * (np.abs(A64) @ np.abs(B64).T) + 1e-5
    err = np.abs(out - ref)
    assert (err <= bound).all(), f"max err {err.max()}, worst ratio {(err / bound).max()}"


@pytest.mark.parametrize("M,N,K", [(3005, 1280, 1280), (4096, 1280, 5120), (2053, 1088, 1280), (1500, 512, 2048),
                                   (128, 1280, 5120), (37, 384, 1536)])
def test_gemm_resid_epilogue(wrs, ctx, M, N, K):
    """EPI_RESID (x += A.B^T + bias, f32 residual in place) on the big-tile path (prefetched residual
    loads) and the decode path, with a random initial residual and ragged M / N edges."""
    L = wrs.lib()
    rng = np.random.default_rng(M + 3 * N + K)
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    x0 = rng.standard_normal((M, N)).astype(np.float32)
    pa, pb, pbias, px = _dev(wrs, ctx, A), _dev(wrs, ctx, B), _dev(wrs, ctx, bias), _dev(wrs, ctx, x0)
    ms = C.c_float()
    assert L.whisper_mi355x_debug_gemm(ctx.ptr, 2, C.c_void_p(pa), M, K, C.c_void_p(pb), N, C.c_void_p(pbias),
                                       C.c_void_p(px), 0, C.byref(ms)) == 0
    out = np.empty_like(x0)
    L.whisper_mi355x_memcpy(ctx.ptr, out.ctypes.data, C.c_void_p(px), out.nbytes, 2)
    for p in (pa, pb, pbias, px):
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    ref = x0 + A64 @ B64.T + bias
    bound = 1e-4 * (np.abs(A64) @ np.abs(B64).T) + 1e-5 + 1e-6 * np.abs(x0)
    err = np.abs(out - ref)
    assert (err <= bound).all(), f"max err {err.max()}, worst ratio {(err / bound).max()}"


@pytest.mark.parametrize("M,N,K", [(1, 1280, 1280), (37, 384, 1536), (128, 1280, 5120), (128, 1280, 1280), (64, 1024, 4096)])
def test_gemm_resid_ln_matches_numpy(wrs, ctx, M, N, K):
    """Decode-step residual GEMM + fused LayerNorm (split-K slabs -> reduce + residual + LN)."""
    L = wrs.lib()
    L.whisper_mi355x_debug_gemm_ln.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                               C.POINTER(C.c_float)]
    rng = np.random.default_rng(M * 3 + N + K)
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    x = rng.standard_normal((M, N)).astype(np.float32)
    w = (1.0 + 0.1 * rng.standard_normal(N)).astype(np.float32)
    b = (0.1 * rng.standard_normal(N)).astype(np.float32)
    y = np.zeros((M, N), np.float16)
    ptrs = [_dev(wrs, ctx, a) for a in (A, B, bias, x, w, b, y)]
    ms = C.c_float()
    assert L.whisper_mi355x_debug_gemm_ln(ctx.ptr, C.c_void_p(ptrs[0]), M, K, C.c_void_p(ptrs[1]), N, C.c_void_p(ptrs[2]),
                                          C.c_void_p(ptrs[3]), C.c_void_p(ptrs[4]), C.c_void_p(ptrs[5]),
                                          C.c_void_p(ptrs[6]), 1, C.byref(ms)) == 0
    xo = np.empty_like(x)
    L.whisper_mi355x_memcpy(ctx.ptr, xo.ctypes.data, C.c_void_p(ptrs[3]), xo.nbytes, 2)
    L.whisper_mi355x_memcpy(ctx.ptr, y.ctypes.data, C.c_void_p(ptrs[6]), y.nbytes, 2)
    for p in ptrs:
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
    A64, B64 = A.astype(np.float64), B.astype(np.float64)
    xr = x + A64 @ B64.T + bias
    bound = 1e-4 * (np.abs(A64) @ np.abs(B64).T) + 1e-5 + 1e-6 * np.abs(xr)
    assert (np.abs(xo - xr) <= bound).all(), f"residual max err {np.abs(xo - xr).max()}"
    mu = xr.mean(1, keepdims=True)
    var = ((xr - mu) ** 2).mean(1, keepdims=True)
    yr = (xr - mu) / np.sqrt(var + 1e-5) * w + b
    err = np.abs(y.astype(np.float64) - yr)
    assert (err <= 2e-3 + 2e-3 * np.abs(yr)).all(), f"LN max err {err.max()}"


def _gelu_ggml(x):
    """ggml_vec_gelu_f32 under GGML_GELU_FP16 (the oracle's gelu_ggml, oracle/oracle_whisper.cpp:253):
    |x| >= 10 shortcuts, else table[f16(x)], the table built with libm's tanhf in f32 arithmetic."""
    libm = C.CDLL("libm.so.6")
    libm.tanhf.restype, libm.tanhf.argtypes = C.c_float, [C.c_float]
    h = np.arange(65536, dtype=np.uint32).astype(np.uint16).view(np.float16).astype(np.float32)
    f = np.float32
    with np.errstate(all="ignore"):
        arg = (f(0.7978845608028654) * h) * (f(1) + (f(0.044715) * h) * h)
        t = np.array([libm.tanhf(float(v)) for v in arg], np.float32)
        table = ((f(0.5) * h) * (f(1) + t)).astype(np.float16)
    g = table[x.astype(np.float16).view(np.uint16)]
    return np.where(x <= -10, np.float16(0), np.where(x >= 10, x.astype(np.float16), g))


@pytest.mark.parametrize("M,N,K", [(3000, 1536, 384), (64, 1536, 384), (1, 5120, 1280)])
def test_gemm_gelu_epilogue(wrs, ctx, M, N, K):
    """The GELU epilogue (ggml's f16 GELU table, built on the host and uploaded) against the same
    GEMM's f32 output through a numpy restatement of that table, bit for bit; the pre-activations
    straddle the +-10 shortcuts (values in (-10, 10) that round to +-10 in f16 use the table)."""
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.linspace(-12.0, 12.0, N).astype(np.float32)
    pre, _ = _run_gemm(wrs, ctx, A, B, bias, -1, epi=4)
    got, _ = _run_gemm(wrs, ctx, A, B, bias, -1, epi=1)
    ref = _gelu_ggml(pre)
    same = (got.view(np.uint16) == ref.view(np.uint16)) | (got.astype(np.float32) == ref.astype(np.float32))
    assert same.all(), f"{(~same).sum()} of {same.size} differ, e.g. pre {pre[~same][:4]} got {got[~same][:4]} ref {ref[~same][:4]}"


@pytest.mark.parametrize("M,N,K,epi,lna", [(1, 1280, 1280, 4, True), (16, 3840, 1280, 4, True), (32, 1280, 1280, 2, False),
                                           (17, 1280, 5120, 2, False), (7, 5120, 1280, 4, True), (32, 384, 1536, 4, False),
                                           (3, 1536, 512, 4, True)])
def test_gemm_small_matches_numpy(wrs, ctx, M, N, K, epi, lna):
    """Decode steps of <= 32 rows (gemm_small_kernel: 16 columns per workgroup over the whole K, the
    8 waves' partial sums added in LDS; no split-K slabs): f32 output (epi 4) or the residual add (epi
    2), and with lna the LayerNorm of the f32 input rows applied in the prologue (ggml_norm, rounded
    to the MFMA type like the split-K path's fused reduce + LN)."""
    L = wrs.lib()
    L.whisper_mi355x_debug_gemm_small.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                                  C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                                  C.POINTER(C.c_float)]
    rng = np.random.default_rng(M * 11 + N + K)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    w = (1.0 + 0.1 * rng.standard_normal(K)).astype(np.float32)
    b = (0.1 * rng.standard_normal(K)).astype(np.float32)
    if lna:
        X = (3.0 * rng.standard_normal((M, K)) + 0.5).astype(np.float32)
        mu = X.astype(np.float64).mean(1, keepdims=True)
        var = ((X.astype(np.float64) - mu) ** 2).mean(1, keepdims=True)
        A64 = ((X - mu) / np.sqrt(var + 1e-5) * w + b).astype(np.float16).astype(np.float64)
        A = X
    else:
        A = rng.standard_normal((M, K)).astype(np.float16)
        A64 = A.astype(np.float64)
    x0 = rng.standard_normal((M, N)).astype(np.float32)
    out = x0.copy() if epi == 2 else np.zeros((M, N), np.float32)
    ptrs = [_dev(wrs, ctx, a) for a in (A, B, bias, out, w, b)]
    ms = C.c_float()
    assert L.whisper_mi355x_debug_gemm_small(ctx.ptr, epi, C.c_void_p(ptrs[0]), M, K, C.c_void_p(ptrs[1]), N,
                                             C.c_void_p(ptrs[2]), C.c_void_p(ptrs[3]),
                                             C.c_void_p(ptrs[4]) if lna else None, C.c_void_p(ptrs[5]) if lna else None,
                                             0, C.byref(ms)) == 0
    L.whisper_mi355x_memcpy(ctx.ptr, out.ctypes.data, C.c_void_p(ptrs[3]), out.nbytes, 2)
    for p in ptrs:
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
    B64 = B.astype(np.float64)
    ref = A64 @ B64.T + bias + (x0 if epi == 2 else 0.0)
    # lna: an operand rounded one f16 ulp differently from numpy's LN moves a product by <= 2^-10 |a b|
    bound = (2e-3 if lna else 1e-4) * (np.abs(A64) @ np.abs(B64).T) + 1e-5 + 1e-6 * np.abs(ref)
    err = np.abs(out - ref)
    assert (err <= bound).all(), f"max err {err.max()}, worst ratio {(err / bound).max()}"


def _to_bf16_bits(x):
    """float32 -> bf16 bit patterns (round to nearest even), and their float32 values"""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r, (r.astype(np.uint32) << 16).view(np.float32)


def _attn_run(wrs, ctx, qkv_dev, B, T, d, H, variant, reps=0):
    L = wrs.lib()
    L.whisper_mi355x_debug_attn_encoder.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                                    C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_float)]
    out = np.zeros((B * T, d), np.uint16)
    po = _dev(wrs, ctx, out)
    ms = C.c_float()
    assert L.whisper_mi355x_debug_attn_encoder(ctx.ptr, C.c_void_p(qkv_dev), B, T, d, H, variant, C.c_void_p(po),
                                               reps, C.byref(ms)) == 0
    L.whisper_mi355x_memcpy(ctx.ptr, out.ctypes.data, C.c_void_p(po), out.nbytes, 2)
    L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(po))
    return out, ms.value


@pytest.mark.parametrize("dtype,B,T,H", [("BF16", 2, 1500, 20), ("F16", 3, 1500, 6), ("BF16", 1, 100, 8),
                                         ("F16", 2, 64, 4)])
def test_attn_encoder_pipelined_equals_enc2(wrs, micro_model, dtype, B, T, H):
    """Every encoder-attention variant == attn_enc2_kernel bit for bit (same per-element operations and
    order): 3 = score MFMAs of the next key tile issued under the softmax of the current one, 5 = variant 2
    held to 128 VGPRs (two workgroups per CU), 6 = 5 with scalar instead of packed f32 exponent arguments
    and row sums (the default); and variant 2 against a float64
    softmax(Q K^T / 8) V of the same rounded operands."""
    c = wrs.WhisperContext(micro_model, dtype=getattr(wrs, dtype))
    d = 64 * H
    rng = np.random.default_rng(B * 1000 + T + H)
    x = rng.standard_normal((B * T, 3 * d), dtype=np.float32) * 1.5
    if dtype == "BF16":
        bits, xv = _to_bf16_bits(x)
    else:
        h = x.astype(np.float16)
        bits, xv = h.view(np.uint16), h.astype(np.float32)
    L = wrs.lib()
    p = _dev(wrs, c, np.ascontiguousarray(bits))
    o2, _ = _attn_run(wrs, c, p, B, T, d, H, 2)
    bad = {}
    for v in (3, 5, 6):  # every variant: the same per-element operations in the same order
        ov, _ = _attn_run(wrs, c, p, B, T, d, H, v)
        if not np.array_equal(o2, ov):
            bad[v] = int((o2 != ov).sum())
    assert not bad, bad
    L.whisper_mi355x_dev_free(c.ptr, C.c_void_p(p))
    c.close()
    val = ((o2.astype(np.uint32) << 16).view(np.float32) if dtype == "BF16" else o2.view(np.float16).astype(np.float32))
    q, k, v = (xv[:, :d].reshape(B, T, H, 64), xv[:, d:2 * d].reshape(B, T, H, 64), xv[:, 2 * d:].reshape(B, T, H, 64))
    for bb in range(B):
        for hh in range(0, H, max(1, H // 3)):
            s = q[bb, :, hh].astype(np.float64) @ k[bb, :, hh].astype(np.float64).T / 8.0
            pm = np.exp(s - s.max(1, keepdims=True))
            ref = (pm / pm.sum(1, keepdims=True)) @ v[bb, :, hh].astype(np.float64)
            got = val.reshape(B, T, H, 64)[bb, :, hh]
            tol = (2e-2 if dtype == "BF16" else 4e-3) * np.abs(v[bb, :, hh]).max()
            assert np.abs(got - ref).max() <= tol, (bb, hh, np.abs(got - ref).max(), tol)


def test_attn_encoder_variant_timing(wrs, micro_model):
    """large-v3 shape, one 32-window launch (the engine's encoder group): time every variant."""
    c = wrs.WhisperContext(micro_model, dtype=wrs.BF16)
    B, T, H = 32, 1500, 20
    d = 64 * H
    rng = np.random.default_rng(5)
    bits, _ = _to_bf16_bits(rng.standard_normal((B * T, 3 * d), dtype=np.float32))
    L = wrs.lib()
    p = _dev(wrs, c, bits)
    flop = 4.0 * B * H * T * T * 64
    ref = None
    line = []
    for v in (2, 3, 5, 6, 2, 5, 6):
        o, ms = _attn_run(wrs, c, p, B, T, d, H, v, reps=5)
        line.append(f"v{v} {ms * 1e3:.1f} us {flop / ms / 1e9:.0f} TF/s")
        ref = o if ref is None else ref
        assert np.array_equal(o, ref), v
    L.whisper_mi355x_dev_free(c.ptr, C.c_void_p(p))
    c.close()
    print("attn_encoder 32 x 1500 x 20 heads: " + ", ".join(line))


@pytest.mark.parametrize("M", [1, 16, 32, 33, 64, 100])
def test_dec_gemm_row_tiles_bitwise(wrs, micro_model, M):
    """The split-K decode GEMM's row tile (32 / 64 / 128 rows, gemm.hip launch_dec) changes no output bit:
    every output keeps its k order. Large-v3 decode shapes, f16 and bf16, store / GELU / f32 epilogues; the
    128-row tile (whisper_mi355x_set_dec_bm(128)) against the default (the smallest tile holding M rows)."""
    L = wrs.lib()
    L.whisper_mi355x_set_dec_bm.argtypes = [C.c_int]
    for dt in (wrs.F16, wrs.BF16):
        c = wrs.WhisperContext(micro_model, dtype=dt)
        try:
            for (N, K, epi) in [(3840, 1280, 4), (1280, 1280, 0), (5120, 1280, 1), (1280, 5120, 4)]:
                rng = np.random.default_rng(M * 31 + N + K)
                A = rng.standard_normal((M, K)).astype(np.float16)
                B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
                bias = (0.1 * rng.standard_normal(N)).astype(np.float32)
                outs = []
                for bm in (128, 0):
                    L.whisper_mi355x_set_dec_bm(bm)
                    try:
                        outs.append(_run_gemm(wrs, c, A, B, bias, -1, epi=epi)[0])
                    finally:
                        L.whisper_mi355x_set_dec_bm(0)
                assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8)), (dt, N, K, epi)
                assert np.isfinite(outs[1].astype(np.float32)).all()
        finally:
            c.close()
