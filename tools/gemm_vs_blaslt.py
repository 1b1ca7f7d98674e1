"""GPU: the engine's encoder GEMM (bf16, store epilogue) against torch.matmul (hipBLASLt) on the
large-v3 encoder shapes (B windows x 1500 rows): TFLOP/s of each, same operands."""
import ctypes as C
import os
import sys
import time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
ctx = wrs.WhisperContext(model_path("micro"), dtype=wrs.BF16)
rng = np.random.default_rng(0)
d = 1280
B_WIN = int(os.environ.get("B_WIN", "32"))
for (M, N, K, name, epi) in [(B_WIN * 1500, 3 * d, d, "qkv", 0), (B_WIN * 1500, d, d, "out", 2),
                             (B_WIN * 1500, 4 * d, d, "fc1", 1), (B_WIN * 1500, d, 4 * d, "fc2", 2),
                             (B_WIN * 1500, 4 * d, d, "fc1-gelu_f", 7), (B_WIN * 1500, 4 * d, d, "fc1-store", 0)]:
    A = rng.standard_normal((M, K)).astype(np.float16)
    B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    res = []
    for v in [int(x) for x in os.environ.get("VARIANTS", "-1").split(",")]:
        _, msv = _run_gemm(wrs, ctx, A, B, bias, v, reps=5, epi=epi)
        res.append(f"v{v} {2.0 * M * N * K / msv / 1e9:.0f}")
    ms = msv
    ta = torch.from_numpy(A).to(torch.bfloat16).cuda()
    tb = torch.from_numpy(B).to(torch.bfloat16).cuda()
    for _ in range(3):
        torch.matmul(ta, tb.t())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch.matmul(ta, tb.t())
    e1.record()
    torch.cuda.synchronize()
    tms = e0.elapsed_time(e1) / 10
    f = 2.0 * M * N * K

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 10

    # the same epilogue through hipBLASLt where torch exposes it: f32 residual C = D (beta = 1) for epi 2,
    # the bias + GELU epilogue for epi 1
    fair = ""
    try:
        if epi == 2:
            resid = torch.zeros((M, N), dtype=torch.float32, device="cuda")
            t2 = timed(lambda: torch.addmm(resid, ta, tb.t(), out_dtype=torch.float32))
            fair = f" | hipBLASLt f32 C+=AB {t2:.3f} ms {f / t2 / 1e9:.0f} TF/s"
        elif epi in (1, 7):
            bb = torch.zeros(N, dtype=torch.bfloat16, device="cuda")
            t2 = timed(lambda: torch._addmm_activation(bb, ta, tb.t(), use_gelu=True))
            fair = f" | hipBLASLt bias+GELU {t2:.3f} ms {f / t2 / 1e9:.0f} TF/s"
    except Exception as ex:  # noqa: BLE001
        fair = f" | fair variant unavailable: {type(ex).__name__}: {str(ex)[:80]}"
    print(f"{name:9s} M={M} N={N} K={K}: engine epi{epi} [{', '.join(res)}] TF/s | hipBLASLt {tms:.3f} ms "
          f"{f / tms / 1e9:.0f} TF/s{fair}", flush=True)
