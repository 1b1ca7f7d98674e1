"""Time the per-layer cross K/V GEMM shape (M = 128 x 1500, N = 2 d, K = d, large-v3) with a plain contiguous store
epilogue, to compare with the EPI_CROSSKV launch (rocprof: ~2.6 ms per layer at 128 clips)."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from test_gpu_kernels import _run_gemm

wrs = load_whisper_rs()
rng = np.random.default_rng(0)
ctx = wrs.WhisperContext(model_path("large-v3-2L"), dtype=wrs.BF16)  # n_audio_ctx 1500 (EPI_CROSSKV's row blocks)
for (M, N, K, name, epi) in [(128 * 1500, 2560, 1280, "xkv-layer store", 0), (128 * 1500, 2560, 1280, "xkv-layer crosskv", 5),
                             (128 * 1500, 2560 * 4, 1280, "xkv-4layers crosskv", 5), (128 * 1500, 3840, 1280, "qkv store", 0)]:
    A = (rng.standard_normal((M, K), dtype=np.float32)).astype(np.float16)
    B = (rng.standard_normal((N, K), dtype=np.float32) / np.sqrt(K)).astype(np.float16)
    bias = np.zeros(N, np.float32)
    _, ms = _run_gemm(wrs, ctx, A, B, bias, -1, reps=5, epi=epi)
    print(f"{name} M={M} N={N} K={K}: {ms * 1e3:.0f} us, {2.0 * M * N * K / ms / 1e9:.0f} TF/s", flush=True)
ctx.close()
