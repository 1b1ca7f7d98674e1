"""GPU: time of the direct cross-attention kernels (Q' projection + step + combine, debug hook) on the
large-v3 decode shape: n tokens (one clip each) x 1500 encoder rows x d, and the HBM rate on E.
SAMESLOT=1: every clip reads the same E (cache-resident): the kernel's rate without the HBM stream."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path

wrs = load_whisper_rs()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
L = wrs.lib()
L.whisper_mi355x_debug_xattn.argtypes = [C.c_void_p] * 7 + [C.c_int] * 3 + [C.c_float, C.c_int, C.c_float, C.c_void_p,
                                                                             C.c_int, C.POINTER(C.c_float)]
d, Tn = int(os.environ.get("D", "1280")), 1500
H = d // 64
rng = np.random.default_rng(0)
for n in [int(x) for x in os.environ.get("NS", "128,64").split(",")]:
    arrs = [(rng.standard_normal((n, Tn, d)) * 0.5).astype(np.float16).view(np.uint16), (np.zeros(n, np.int32) if os.environ.get("SAMESLOT") else np.arange(n, dtype=np.int32)),
            rng.standard_normal((n, d)).astype(np.float16).view(np.uint16),
            (rng.standard_normal((H, d, 64)) / 30).astype(np.float16).view(np.uint16),
            (rng.standard_normal((d, d)) / 30).astype(np.float16).view(np.uint16), np.zeros(d, np.float32)]
    ptrs = []
    for a in arrs:
        p = L.whisper_mi355x_dev_alloc(ctx.ptr, a.nbytes)
        L.whisper_mi355x_memcpy(ctx.ptr, C.c_void_p(p), a.ctypes.data, a.nbytes, 1)
        ptrs.append(p)
    po = L.whisper_mi355x_dev_alloc(ctx.ptr, n * d * 2)
    for sp in [int(x) for x in os.environ.get("SPLITS", "0").split(",")]:  # 0 = the engine's choice
        ms = C.c_float()
        assert L.whisper_mi355x_debug_xattn(ctx.ptr, *[C.c_void_p(p) for p in ptrs], n, Tn, d, 64 ** -0.25, sp, 8.0,
                                            C.c_void_p(po), 20, C.byref(ms)) == 0
        out = np.zeros(n * d, np.uint16)
        L.whisper_mi355x_memcpy(ctx.ptr, out.ctypes.data, C.c_void_p(po), out.nbytes, 2)
        import hashlib
        print(f"n={n} d={d} splits={sp} {ms.value * 1e3:.1f} us per call "
              f"(qproj+step+combine), E {n * Tn * d * 2 / (ms.value * 1e-3) / 1e9:.0f} GB/s (whole call) "
              f"out {hashlib.sha1(out.tobytes()).hexdigest()[:12]}", flush=True)
    for p in ptrs + [po]:
        L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(p))
