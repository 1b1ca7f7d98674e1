"""GPU: TFLOP/s of the engine's GEMM on the large-v3 encoder shapes (B windows x 1500 rows), per
epilogue (0 store, 1 GELU, 2 f32 residual) and variant (-1 = the engine's choice)."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16 if "--bf16" in sys.argv else wrs.F16)
rng = np.random.default_rng(0)
d = 1280
B_WIN = int(os.environ.get("B_WIN", "32"))
variants = [int(v) for v in os.environ.get("VARIANTS", "-1").split(",")]
for (M, N, K, name, epis) in [(B_WIN * 1500, 3 * d, d, "qkv", (0,)), (B_WIN * 1500, d, d, "out", (2,)),
                              (B_WIN * 1500, 4 * d, d, "fc1", (0, 1)), (B_WIN * 1500, d, 4 * d, "fc2", (2,))]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    for epi in epis:
        for v in variants:
            _, ms = _run_gemm(wrs, ctx, A, B, bias, v, reps=5, epi=epi)
            print(f"{name:4s} epi={epi} M={M} N={N} K={K} variant={v}: {ms:.3f} ms  {2.0 * M * N * K / ms / 1e9:.0f} TFLOP/s",
                  flush=True)
