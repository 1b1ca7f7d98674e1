"""Where the encoder GEMM's time goes (gemm.hip gemm8p_kernel debug stamps, whisper_mi355x_set_gemm_stamps):
one launch per large-v3 encoder shape (32 windows x 1500 rows, random bf16 operands); per workgroup the shader
clock at entry, main-loop start, main-loop end and epilogue end. Prints medians of the prologue (entry -> loop),
main loop and epilogue, the loop's cycles per K-tile against the MFMA floor (2048 cycles per 256 x 256 x 64 K-tile per
CU at 4096 bf16 FLOP per cycle). fc1 runs the bf16 engine's GELU-by-formula epilogue (7). usage: python tools/gemm_stamps.py [gemm variant, default -1 = auto]"""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
L = wrs.lib()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
rng = np.random.default_rng(0)
d, M = 1280, 32 * 1500
variant = int(sys.argv[1]) if len(sys.argv) > 1 else -1
for (N, K, name, epi) in [(3 * d, d, "qkv", 0), (d, d, "out", 2), (4 * d, d, "fc1", 7), (d, 4 * d, "fc2", 2)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    grid = ((N + 255) // 256) * ((M + 255) // 256)
    buf = L.whisper_mi355x_dev_alloc(ctx.ptr, grid * 4 * 8)
    _run_gemm(wrs, ctx, A, B, bias, variant, reps=2, epi=epi)  # warm (clocks up)
    L.whisper_mi355x_set_gemm_stamps(C.c_void_p(buf))
    _, ms = _run_gemm(wrs, ctx, A, B, bias, variant, reps=1, epi=epi)
    L.whisper_mi355x_set_gemm_stamps(None)
    st = np.zeros((grid, 4), np.uint64)
    L.whisper_mi355x_memcpy(ctx.ptr, st.ctypes.data, C.c_void_p(buf), st.nbytes, 2)
    L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(buf))
    st = st.astype(np.int64)
    pro, loop, epi_c = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    nk = K // 64
    print(f"{name:4s} N={N} K={K} grid={grid}: {ms * 1e3:.0f} us; per WG median prologue {np.median(pro):.0f} cyc, "
          f"loop {np.median(loop):.0f} cyc ({np.median(loop) / nk:.0f} per K-tile, floor 2048), epilogue "
          f"{np.median(epi_c):.0f} cyc; WG total {np.median(st[:, 3] - st[:, 0]):.0f}", flush=True)
ctx.close()
