"""GPU: TFLOP/s of the fp8 (e4m3, per-row scales, block-scaled MFMA at scale 1) encoder GEMM vs the
bf16 kernel on the large-v3 encoder shapes (B_WIN windows x 1500 rows)."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm
from test_gpu_fp8 import _dev

wrs = load_whisper_rs()
L = wrs.lib()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
L.whisper_mi355x_debug_gemm_fp8.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                            C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                            C.POINTER(C.c_float)]
rng = np.random.default_rng(0)
d = 1280
B_WIN = int(os.environ.get("B_WIN", "32"))
for (M, N, K, name, epi) in [(B_WIN * 1500, 3 * d, d, "qkv", 0), (B_WIN * 1500, 4 * d, d, "fc1", 1),
                             (B_WIN * 1500, d, 4 * d, "fc2", 2), (B_WIN * 1500, d, d, "out", 2)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    _, ms = _run_gemm(wrs, ctx, A, B, bias, -1, reps=5, epi=epi)
    A8 = rng.integers(0, 0x7e, (M, K), dtype=np.uint8)
    B8 = rng.integers(0, 0x7e, (N, K), dtype=np.uint8)
    sa, sb = np.full(M, 1e-3, np.float32), np.full(N, 1e-3, np.float32)
    out = np.zeros((M, N), np.float32 if epi == 2 else np.uint16)
    ptrs = [_dev(L, ctx, a) for a in (A8, sa, B8, sb, bias, out)]
    ms8 = C.c_float()
    assert L.whisper_mi355x_debug_gemm_fp8(ctx.ptr, epi, *[C.c_void_p(p) for p in ptrs[:2]], M, K, C.c_void_p(ptrs[2]),
                                           C.c_void_p(ptrs[3]), N, C.c_void_p(ptrs[4]), C.c_void_p(ptrs[5]), 5,
                                           C.byref(ms8)) == 0
    for p in ptrs:
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
    f = 2.0 * M * N * K / 1e9
    print(f"{name:4s} epi={epi} M={M} N={N} K={K}: bf16 {ms:.3f} ms {f / ms:.0f} TF/s | fp8 {ms8.value:.3f} ms "
          f"{f / ms8.value:.0f} TF/s | x{ms / ms8.value:.2f}", flush=True)
