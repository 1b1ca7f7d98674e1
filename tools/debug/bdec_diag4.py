"""The head of layer 0 of one decode step (embedding -> QKV -> self attention over the prompt's cache ->
out-projection + residual -> LN -> cross q) in numpy from the oracle's weights, against the batched chain's
cross-q rows (debug aid for kernels/bdec.hip)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

from conftest import load_whisper_rs, model_path  # noqa: E402
from make_model import synthetic_pcm  # noqa: E402
from oracle_py import Oracle, reference_params  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "small-1L+conf"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
NT = 2
wrs = load_whisper_rs()
path = model_path(shape)
o = Oracle(path, mode=1, n_threads=16)
ref = o.full(synthetic_pcm(0), reference_params("en", fixed_tokens=NT))
forced = np.array([ref["step_tokens"]] * n, np.int32)
d, H = o.d, o.n_head
f16 = lambda a: np.asarray(a, np.float32).astype(np.float16).astype(np.float64)  # noqa: E731
T = lambda name: o.tensor(name).astype(np.float64)  # noqa: E731


def ln(x, w, b):
    x = np.asarray(x, np.float32)
    mean = np.float32(x.astype(np.float64).sum() / x.size)
    xc = (x - mean).astype(np.float32)
    var = np.float32((xc.astype(np.float64) ** 2).sum() / x.size)
    return (xc * np.float32(1.0 / np.sqrt(var + 1e-5))) * np.float32(w) + np.float32(b)


te = o.tensor("decoder.token_embedding.weight").reshape(-1, d)
pe = o.tensor("decoder.positional_embedding").reshape(-1, d)
sot = o.token("sot")
toks = [sot, sot + 1, o.token("transcribe"), int(forced[0][0])]
W = lambda p: T(f"decoder.blocks.0.{p}.weight").reshape(d, -1)  # noqa: E731
B = lambda p: T(f"decoder.blocks.0.{p}.bias")  # noqa: E731
ks = (d // H) ** -0.25
K, Vv = [], []
for pos, tk in enumerate(toks):
    x = te[tk].astype(np.float32) + pe[pos].astype(np.float32)
    h = f16(ln(x, o.tensor("decoder.blocks.0.attn_ln.weight"), o.tensor("decoder.blocks.0.attn_ln.bias")))
    q = f16((W("attn.query") @ h + B("attn.query")) * ks)
    K.append(f16((W("attn.key") @ h) * ks))
    Vv.append(f16(W("attn.value") @ h + B("attn.value")))
K, Vv = np.stack(K), np.stack(Vv)
att = np.zeros(d)
for hh in range(H):
    sl = slice(hh * 64, hh * 64 + 64)
    s = K[:, sl] @ q[sl]
    p = np.exp(s - s.max())
    p = f16(p / p.sum())
    att[sl] = p @ Vv[:, sl]
att = f16(att)
x1 = (te[toks[3]].astype(np.float64) + pe[3]) + (W("attn.out") @ att + B("attn.out"))
hx = f16(ln(x1, o.tensor("decoder.blocks.0.cross_attn_ln.weight"), o.tensor("decoder.blocks.0.cross_attn_ln.bias")))
xq = f16((W("cross_attn.query") @ hx + B("cross_attn.query")) * ks)

os.environ["WHISPER_MI355X_CROSS"] = "direct"
os.environ["WHISPER_MI355X_BDEC"] = sys.argv[3] if len(sys.argv) > 3 else "1"
os.environ["WHISPER_MI355X_BDEC_HEAD_ONLY"] = "2"  # the step's buffers then hold the head's att / x / cross q
ctx = wrs.WhisperContext(path, dtype=wrs.F16)
st = ctx.create_state()
V = wrs.lib().whisper_n_vocab(ctx.ptr)
rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(0)] * n, NT, forced, [0], V)
L = wrs.lib()
g = np.empty(n * d, np.float16)
L.whisper_mi355x_memcpy(ctx.ptr, g.ctypes.data, L.whisper_mi355x_debug_ws(st.ptr, 5), g.nbytes, 2)
g = g.reshape(n, d).astype(np.float64)
print("xq: max|gpu - numpy|", np.abs(g[0] - xq).max(), " max|numpy|", np.abs(xq).max())
print("  gpu[:8]  ", np.round(g[0][:8], 4))
print("  numpy[:8]", np.round(xq[:8], 4))
a = np.empty(n * d, np.float16)
L.whisper_mi355x_memcpy(ctx.ptr, a.ctypes.data, L.whisper_mi355x_debug_ws(st.ptr, 3), a.nbytes, 2)
a = a.reshape(n, d).astype(np.float64)
print("att: max|gpu - numpy|", np.abs(a[0] - att).max(), " max|numpy|", np.abs(att).max())
print("  gpu[:8]  ", np.round(a[0][:8], 4), " numpy[:8]", np.round(att[:8], 4))
bad = np.nonzero(np.abs(a[0] - att) > 0.02)[0]
print("  bad att columns", len(bad), bad[:24])
xx = np.empty(n * d, np.float32)
L.whisper_mi355x_memcpy(ctx.ptr, xx.ctypes.data, L.whisper_mi355x_debug_ws(st.ptr, 0), xx.nbytes, 2)
xx = xx.reshape(n, d).astype(np.float64)
print("x1: max|gpu - numpy|", np.abs(xx[0] - x1).max(), " max|numpy|", np.abs(x1).max())
print("  gpu[:8]  ", np.round(xx[0][:8], 4), " numpy[:8]", np.round(x1[:8], 4))
bad = np.nonzero(np.abs(xx[0] - x1) > 0.02)[0]
print("  bad x1 columns", len(bad), bad[:24])

hh = np.empty(n * d, np.float16)
L.whisper_mi355x_memcpy(ctx.ptr, hh.ctypes.data, L.whisper_mi355x_debug_ws(st.ptr, 2), hh.nbytes, 2)
hh = hh.reshape(n, d).astype(np.float64)
print("H4 operand (LN(x1)): max|gpu - numpy|", np.abs(hh[0] - hx).max(), " max|numpy|", np.abs(hx).max())
print("  gpu[:8]  ", np.round(hh[0][:8], 4), " numpy[:8]", np.round(hx[:8], 4))
