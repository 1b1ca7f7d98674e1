"""Per-phase timeline of the batched decoder chain (kernels/bdec.hip) from its debug clock stamps.

Every workgroup writes the 100 MHz clock when a phase's input arrived (its wait returned) and when it
published its output; the last decode step's stamps are summarised per phase over the middle launches:
  work    median over WGs of (publish - input)            the phase's own compute
  skew    max - min over WGs of the publish time          load imbalance / stragglers
  hand    min over WGs of the next input - max publish    hand-off latency (last producer -> first consumer)
  gap     between launches: first T1 input - last H5 publish of the previous launch (the E pass between)
usage: python tools/bdec_stamps.py [shape] [dtype] [clips] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

PHASES = ["T1 combine", "T2 wxo+x", "T3 ln+fc1", "T4 fc2+x", "H1 ln+qkv", "H2 self", "H3 wo+x", "H4 ln+xq", "H5 q'"]
NPH = 9


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "large-v3+conf"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "BF16"
    n_clips = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    n_tok = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    os.environ.setdefault("WHISPER_MI355X_CROSS", "direct")
    os.environ.setdefault("WHISPER_MI355X_BDEC", "1")
    from conftest import load_whisper_rs, model_path
    wrs = load_whisper_rs()
    from make_model import synthetic_pcm
    L = wrs.lib()
    ctx = wrs.WhisperContext(model_path(shape), dtype=getattr(wrs, dtype))
    nl = L.whisper_model_n_text_layer(ctx.ptr)
    buf = torch.zeros((nl + 1) * 2 * NPH * 256, dtype=torch.int64, device="cuda")
    L.whisper_mi355x_set_pdec_stamps(C.c_void_p(buf.data_ptr()))
    st = ctx.create_state()
    V = L.whisper_n_vocab(ctx.ptr)
    forced = np.full((n_clips, n_tok), 50364, np.int32)  # the first timestamp token, every step
    rc, _ = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(c % 64) for c in range(n_clips)],
                                 n_tok, forced, [0], V)
    assert rc == 0, rc
    torch.cuda.synchronize()
    L.whisper_mi355x_set_pdec_stamps(None)
    s = buf.cpu().numpy().reshape(nl + 1, 2, NPH, 256).astype(np.float64) * 10.0  # ns
    if not s.any():
        print("no stamps (chain not taken?)")
        return 1
    s[s == 0] = np.nan
    t0 = np.nanmin(s)
    s -= t0
    tot = np.nanmax(s)
    print(f"{shape} {dtype} {n_clips} clips: step chain span {tot / 1e3:.1f} us over {nl + 1} launches")
    print(f"{'phase':12s} {'work us':>8s} {'skew us':>8s} {'hand us':>8s}")
    mid = range(1, nl)
    sums = np.zeros(3)
    with np.errstate(all="ignore"):
        for p in range(NPH):
            w = np.nanmean([np.nanmedian(s[k, 1, p] - s[k, 0, p]) for k in mid])
            sk = np.nanmean([np.nanmax(s[k, 1, p]) - np.nanmin(s[k, 1, p]) for k in mid])
            h = np.nanmean([np.nanmin(s[k, 0, p + 1]) - np.nanmax(s[k, 1, p]) for k in mid]) if p + 1 < NPH else np.nan
            sums += (w, sk, 0 if np.isnan(h) else h)
            print(f"{PHASES[p]:12s} {w / 1e3:8.2f} {sk / 1e3:8.2f} {h / 1e3:8.2f}")
        gap = np.nanmean([np.nanmin(s[k + 1, 0, 0]) - np.nanmax(s[k, 1, NPH - 1]) for k in range(0, nl)])
        span = np.nanmean([np.nanmax(s[k, 1]) - np.nanmin(s[k, 0]) for k in mid])
    print(f"{'sum':12s} {sums[0] / 1e3:8.2f} {sums[1] / 1e3:8.2f} {sums[2] / 1e3:8.2f}")
    print(f"launch span (first input -> last publish) {span / 1e3:.2f} us; gap between launches {gap / 1e3:.2f} us")
    st.close()
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
