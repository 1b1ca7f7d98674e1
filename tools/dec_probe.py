import ctypes as C, os, sys
import numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _dev
wrs = load_whisper_rs(); L = wrs.lib()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
L.whisper_mi355x_debug_gemm.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_float)]
L.whisper_mi355x_set_dec_splits.argtypes = [C.c_int]
rng = np.random.default_rng(0)
for (M, N, K, sp) in [(128, 1280, 128, 1), (128, 1280, 256, 1), (128, 1280, 1280, 1), (128, 1280, 1280, 8), (16, 1280, 1280, 8), (128, 256, 1280, 1)]:
    A = rng.standard_normal((M, K)).astype(np.float16); B = rng.standard_normal((N, K)).astype(np.float16)
    bias = np.zeros(N, np.float32); out = np.zeros((M, N), np.float32)
    ptrs = [_dev(wrs, ctx, a) for a in (A, B, bias, out)]
    L.whisper_mi355x_set_dec_splits(sp)
    ms = C.c_float()
    L.whisper_mi355x_debug_gemm(ctx.ptr, 4, *[C.c_void_p(p) for p in ptrs[:1]], M, K, C.c_void_p(ptrs[1]), N, C.c_void_p(ptrs[2]), C.c_void_p(ptrs[3]), 100, C.byref(ms))
    print(M, N, K, sp, f"{ms.value*1e3:.2f} us/call", flush=True)
    for p in ptrs: L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
