"""Dump teacher-forced decode logits (spot clips 0 and n-1) of an n-clip batch to gpurun_out/envlg_<tag>.npy, for a
bitwise A/B of engine switches that must not change any bit (run once per setting: the switches are read once per
process). Usage: [WHISPER_MI355X_<SWITCH>=v] python tools/debug/env_logits.py <tag> [n] [cache|direct] [prompt]
             python tools/debug/env_logits.py --compare <tagA> <tagB>"""
import os
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a = np.load(os.path.join("gpurun_out", f"envlg_{sys.argv[2]}.npy"))
    b = np.load(os.path.join("gpurun_out", f"envlg_{sys.argv[3]}.npy"))
    eq = np.array_equal(a.view(np.uint32), b.view(np.uint32))
    print(f"{sys.argv[2]} vs {sys.argv[3]}: logits bitwise equal: {eq}, max |diff| {float(np.abs(a - b).max())}")
    sys.exit(0 if eq else 1)

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "tests"), os.path.join(os.path.dirname(__file__), "..")]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
os.environ["WHISPER_MI355X_CROSS"] = sys.argv[3] if len(sys.argv) > 3 else "cache"
from conftest import load_whisper_rs, model_path  # noqa: E402
from make_model import synthetic_pcm  # noqa: E402

wrs = load_whisper_rs()
ntok = 16
ctx = wrs.WhisperContext(model_path("large-v3-2L+conf"), dtype=wrs.BF16)
st = ctx.create_state()
V = wrs.lib().whisper_n_vocab(ctx.ptr)
forced = np.full((n, ntok), 50364, np.int32)
prm = wrs.reference_full_params("en", wrs.DEFAULT_VOCABULARY if len(sys.argv) > 4 and sys.argv[4] == "prompt" else None)
rc, lg = st.full_batch_forced(prm, [synthetic_pcm(k) for k in range(n)], ntok, forced, [0, n - 1], V)
assert rc == 0
np.save(os.path.join("gpurun_out", f"envlg_{sys.argv[1]}.npy"), lg)
print(sys.argv[1], n, lg.shape, float(np.abs(lg).max()))
