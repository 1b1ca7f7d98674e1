"""Dump teacher-forced decode logits (direct cross form, 64 clips, spot clips 0 and 63) of the library named by
WHISPER_MI355X_LIB to gpurun_out/ab_<tag>.npy: a bitwise A/B of two builds."""
import os
import sys

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "tests"), os.path.join(os.path.dirname(__file__), "..")]
os.environ["WHISPER_MI355X_CROSS"] = "direct"
from conftest import load_whisper_rs, model_path  # noqa: E402
from make_model import synthetic_pcm  # noqa: E402

wrs = load_whisper_rs()
n, ntok = 64, 16
ctx = wrs.WhisperContext(model_path("large-v3-2L+conf"), dtype=wrs.BF16)
st = ctx.create_state()
V = wrs.lib().whisper_n_vocab(ctx.ptr)
forced = np.full((n, ntok), 50364, np.int32)
rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(k) for k in range(n)], ntok, forced, [0, 63], V)
assert rc == 0
np.save(os.path.join("gpurun_out", f"ab_{sys.argv[1]}.npy"), lg)
print(sys.argv[1], lg.shape, float(np.abs(lg).max()))
