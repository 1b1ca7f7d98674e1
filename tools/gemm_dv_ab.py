"""GPU A/B of encoder GEMM variants (gemm.hip gemm8p_kernel; DV_VARIANTS = whisper_mi355x_set_gemm_variant values,
e.g. -1 auto, 14 the transposed-accumulator epilogue): the large-v3 encoder shapes (32 windows x 1500 rows, random
bf16 operands, the engine's epilogues incl. bias), each variant timed over 5 launches in rounds so that clock drift
spreads over all of them; outputs must be bitwise equal across variants."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
rng = np.random.default_rng(0)
d = 1280
M = 32 * 1500
variants = [int(v) for v in os.environ.get("DV_VARIANTS", "-1").split(",")]
for (N, K, name, epi) in [(3 * d, d, "qkv", 0), (d, d, "out", 2), (4 * d, d, "fc1", 7), (d, 4 * d, "fc2", 2),
                          (4 * d, d, "fc1-table", 1), (3 * d, d, "f32", 4)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = rng.standard_normal(N).astype(np.float32)
    t = {v: [] for v in variants}
    outs = {}
    for rnd in range(3):
        for v in variants:
            o, ms = _run_gemm(wrs, ctx, A, B, bias, v, reps=5, epi=epi)
            t[v].append(ms)
            if rnd == 0:
                outs[v] = o
    same = all(np.array_equal(outs[v].view(np.uint8), outs[variants[0]].view(np.uint8)) for v in variants)
    f = 2.0 * M * N * K
    print(f"{name:4s} M={M} N={N} K={K}: " + "  ".join(
        f"v{v} {f / np.median(t[v]) / 1e9:.0f} TF/s ({np.median(t[v]) * 1e3:.0f} us)" for v in variants) +
        f"  bitwise-equal {same}", flush=True)
ctx.close()
