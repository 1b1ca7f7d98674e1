"""GPU: per-call time of the decode-step GEMMs (M = active clips) on large-v3 shapes, per variant and
split count. Times are back-to-back launches on one stream (kernel boundaries included), i.e. what
one decode step pays per GEMM. GB/s = weight bytes / time."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path  # noqa: E402
from test_gpu_kernels import _dev  # noqa: E402

wrs = load_whisper_rs()
L = wrs.lib()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
L.whisper_mi355x_debug_gemm.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_float)]
L.whisper_mi355x_debug_gemm_ln.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_float)]
L.whisper_mi355x_set_gemm_variant.argtypes = [C.c_int]
L.whisper_mi355x_set_dec_splits.argtypes = [C.c_int]
d = 1280
rng = np.random.default_rng(0)
REPS = 200
Ms = [int(x) for x in os.environ.get("DEC_M", "16,128").split(",")]
splits_list = [int(x) for x in os.environ.get("DEC_SPLITS", "0").split(",")]
variants = [int(x) for x in os.environ.get("DEC_VARIANTS", "1").split(",")]  # 1 = split-K + reduce (the decode path)
for M in Ms:
    for (N, K, name, epi) in [(3 * d, d, "qkv", 0), (d, d, "q", 0), (4 * d, d, "fc1", 1), (d, d, "out+ln", -1),
                              (d, 4 * d, "fc2+ln", -1), (51866, d, "logits", 4)]:
        A = rng.standard_normal((M, K)).astype(np.float16)
        B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
        bias = np.zeros(N, np.float32)
        out = np.zeros((M, N), np.float32)
        ln = np.ones(N, np.float32)
        ptrs = [_dev(wrs, ctx, a) for a in (A, B, bias, out, ln, ln, out)]
        for v in variants:
            for sp in splits_list:
                L.whisper_mi355x_set_gemm_variant(v)
                L.whisper_mi355x_set_dec_splits(sp)
                ms = C.c_float()
                if epi < 0:
                    rc = L.whisper_mi355x_debug_gemm_ln(ctx.ptr, C.c_void_p(ptrs[0]), M, K, C.c_void_p(ptrs[1]), N,
                                                        C.c_void_p(ptrs[2]), C.c_void_p(ptrs[3]), C.c_void_p(ptrs[4]),
                                                        C.c_void_p(ptrs[5]), C.c_void_p(ptrs[6]), REPS, C.byref(ms))
                else:
                    rc = L.whisper_mi355x_debug_gemm(ctx.ptr, epi, C.c_void_p(ptrs[0]), M, K, C.c_void_p(ptrs[1]), N,
                                                     C.c_void_p(ptrs[2]), C.c_void_p(ptrs[3]), REPS, C.byref(ms))
                assert rc == 0
                us = ms.value * 1e3
                print(f"M={M:4d} {name:7s} N={N:6d} K={K:5d} variant={v} splits={sp}: {us:8.2f} us "
                      f"{N * K * 2 / us / 1e3:7.0f} GB/s", flush=True)
        L.whisper_mi355x_set_gemm_variant(-1)
        L.whisper_mi355x_set_dec_splits(0)
        for p in ptrs:
            L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
