"""GPU A/B of the decode-step GEMM at 128 rows: the split-K kernel + its reduce launch (variant -1, the engine's
path) against the register-direct full-K kernel (gemm.hip gemm_rowfull_kernel, variants 20 / 21 / 22 = 4 / 6 / 8
K-chunks in flight per lane). Times back-to-back launches (reps) of the large-v3 decode shapes; checks each
variant against float64 numpy on f16 operands (|err| <= 1e-4 * sum |a b| + 1e-3 after the f16 output rounding)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
variants = [int(v) for v in os.environ.get("VARIANTS", "-1,20,21,22").split(",")]
rng = np.random.default_rng(1)
M, d = 128, 1280
ctx16 = wrs.WhisperContext(model_path("micro"), dtype=wrs.F16)
for (N, K, name, epi) in [(4 * d, d, "fc1-gelu", 1), (d, d, "xq-store", 0), (3 * d, d, "qkv-f32", 4)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = (0.1 * rng.standard_normal(N)).astype(np.float32)
    ref = A.astype(np.float64) @ B.astype(np.float64).T + bias
    bound = np.abs(A.astype(np.float64)) @ np.abs(B.astype(np.float64)).T
    line = []
    for v in variants:
        out, _ = _run_gemm(wrs, ctx16, A, B, bias, v, reps=1, epi=epi)
        if epi == 1:
            ok = np.isfinite(out).all()  # GELU output: compare pre-activation only loosely
            err = 0.0
        else:
            err = float(np.max(np.abs(out.astype(np.float64) - ref) - (1e-4 * bound + 2e-3 * np.abs(ref) + 1e-3)))
            ok = err <= 0
        line.append(f"v{v} ok={ok}")
    print(f"{name} numerics: " + " ".join(line), flush=True)
ctx16.close()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
for (N, K, name, epi) in [(4 * d, d, "fc1-gelu", 1), (d, d, "xq-store", 0), (3 * d, d, "qkv-f32", 4), (d, 4 * d, "fc2-f32", 4)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    t = {v: [] for v in variants}
    for rnd in range(3):
        for v in variants:
            _, ms = _run_gemm(wrs, ctx, A, B, bias, v, reps=20, epi=epi)
            t[v].append(ms)
    print(f"{name:9s} M={M} N={N} K={K}: " + "  ".join(f"v{v} {np.median(t[v]) * 1e3:.1f} us" for v in variants), flush=True)
ctx.close()
