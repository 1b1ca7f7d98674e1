"""GPU A/B of the decode-step GEMM row tile (gemm.hip gemm_dec_kernel BM = 32 / 64 vs 128, and 65..128 rows as
two 64-row chunks): run once per WHISPER_MI355X_DEC_BM / _DEC_M64 setting (the value is read once per process), time back-to-back launches of the
large-v3 decode shapes at small step sizes, save the outputs, and with --compare check the two runs'
outputs are bit-identical (the row tile does not change any output's k order).
Usage: WHISPER_MI355X_DEC_BM=128 python tools/dec_bm_ab.py gpurun_out/bm128.npz
       WHISPER_MI355X_DEC_BM=32 python tools/dec_bm_ab.py gpurun_out/bm32.npz
       python tools/dec_bm_ab.py --compare gpurun_out/bm128.npz gpurun_out/bm32.npz"""
import os
import sys
import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8))]
    print("bitwise equal" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
d = 1280
outs = {}
tag = os.environ.get("WHISPER_MI355X_DEC_BM", "auto") + " M64=" + os.environ.get("WHISPER_MI355X_DEC_M64", "0")
for dt_name, dt in (("f16", wrs.F16), ("bf16", wrs.BF16)):
    ctx = wrs.WhisperContext(model_path("micro"), dtype=dt)
    for M in (1, 7, 16, 32, 33, 64, 65, 96, 128):
        line = []
        for (N, K, name, epi) in [(3 * d, d, "qkv", 4), (d, d, "xq", 0), (4 * d, d, "fc1", 1), (d, 4 * d, "fc2", 4)]:
            rng = np.random.default_rng(M * 31 + N + K)
            A = rng.standard_normal((M, K)).astype(np.float16)
            B = (rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float16)
            bias = (0.1 * rng.standard_normal(N)).astype(np.float32)
            out, _ = _run_gemm(wrs, ctx, A, B, bias, -1, reps=1, epi=epi)
            outs[f"{dt_name}_{name}_{M}"] = out
            _, ms = _run_gemm(wrs, ctx, A, B, bias, -1, reps=200, epi=epi)
            line.append(f"{name} {ms * 1e3:6.1f}")
        print(f"BM={tag} {dt_name} M={M:3d}: " + "  ".join(line) + "  (us per call)", flush=True)
    ctx.close()
np.savez(sys.argv[1], **outs)
