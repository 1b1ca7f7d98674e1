"""One decode step of a 1-layer model through the batched chain and through the launch chain: the step's
buffers compared in dependency order (debug aid for kernels/bdec.hip)."""
import ctypes as C
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
NT = 2  # the prefill + one decode step
wrs = load_whisper_rs()
path = model_path(shape)
o = Oracle(path, mode=1, n_threads=16)
ref = o.full(synthetic_pcm(0), reference_params("en", fixed_tokens=NT))
forced = np.array([ref["step_tokens"]] * n, np.int32)
hp = (o.d, o.n_head)
d, H = hp
S = max(1, min(16, (256 + n - 1) // n))
sizes = {0: (n * d, np.float32), 1: (n * d, np.float16), 3: (n * d, np.float16), 4: (n * 4 * d, np.float16),
         5: (n * d, np.float16), 6: (n * 2 * H * d, np.float16), 7: (n * S * H * d, np.float32), 8: (n * S * H * 2, np.float32)}
names = {0: "x", 1: "dh", 3: "att", 4: "ff", 5: "xq", 6: "qx", 7: "xo", 8: "xml"}
got = {}
for b in ("1", "0"):
    os.environ["WHISPER_MI355X_CROSS"] = "direct"
    os.environ["WHISPER_MI355X_BDEC"] = b
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    st = ctx.create_state()
    V = wrs.lib().whisper_n_vocab(ctx.ptr)
    rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(0)] * n, NT, forced, [0], V)
    assert rc == 0
    L = wrs.lib()
    got[b] = {"logits": lg[1, 0, :].copy()}
    for k, (cnt, dtp) in sizes.items():
        p = L.whisper_mi355x_debug_ws(st.ptr, k)
        buf = np.empty(cnt, dtp)
        L.whisper_mi355x_memcpy(ctx.ptr, buf.ctypes.data, p, buf.nbytes, 2)
        got[b][names[k]] = buf.astype(np.float64)
    st.close()
    ctx.close()
print("logits: |bdec - chain| =", np.abs(got["1"]["logits"] - got["0"]["logits"]).max(),
      "| oracle", np.abs(got["0"]["logits"] - ref["step_logits"][1]).max())
for k in ("xq", "qx", "xo", "xml", "att", "ff", "x", "dh"):
    a, b = got["1"][k], got["0"][k]
    print(f"{k:4s}: max|bdec - chain| {np.abs(a - b).max():.5f}  max|chain| {np.abs(b).max():.3f}  "
          f"rows equal {[bool(np.allclose(a.reshape(n, -1)[i], b.reshape(n, -1)[i], atol=1e-2)) for i in range(n)]}")
    print("      bdec row0[:6]", np.round(a.reshape(n, -1)[0][:6], 4), " chain", np.round(b.reshape(n, -1)[0][:6], 4))
