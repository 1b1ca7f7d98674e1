"""whisper_full on the engine vs the oracle, token by token with log-probs and oracle margins:
python tools/debug/full_cmp.py SHAPE CLIP DTYPE [t_inc]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params
wrs = load_whisper_rs()
shape, clip, dt = sys.argv[1], int(sys.argv[2]), getattr(wrs, sys.argv[3])
t_inc = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
pcm = synthetic_pcm(clip)
o = Oracle(model_path(shape), mode=1, n_threads=16)
rp = reference_params("en"); rp.temperature_inc = t_inc
ref = o.full(pcm, rp)
ctx = wrs.WhisperContext(model_path(shape), dtype=dt)
st = ctx.create_state()
gp = wrs.reference_full_params("en"); gp.temperature_inc = t_inc
assert st.full(gp, pcm) == 0
got = [(t[0], t[3]) for s in st.segments() for t in s.tokens]
exp = [t for s in ref["segments"] for t in s["tokens"]]
m = ref["margins"]
print("cross", os.environ.get("WHISPER_MI355X_CROSS"), "n got", len(got), "n exp", len(exp), "n margins", len(m))
for i in range(max(len(got), len(exp))):
    g = got[i] if i < len(got) else None
    e = exp[i] if i < len(exp) else None
    print(i, g, e, "margin %.3f" % m[i] if i < len(m) else "", "" if g and g[0] == e else "<<<")
