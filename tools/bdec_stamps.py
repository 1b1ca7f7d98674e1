"""Per-phase timeline of the batched decoder chain (kernels/bdec.hip) from its debug clock stamps.

Every workgroup writes the 100 MHz clock when a phase's input arrived (its wait returned) and when it
published its output; the last decode step's stamps are summarised per phase over the middle launches:
  work    median over WGs of (publish - input)            the phase's own compute
  operand median over WGs of (operand image in LDS - input) (GEMM phases: the A image load / LayerNorm)
  skew    max - min over WGs of the publish time          load imbalance / stragglers
  hand    min over WGs of the next input - max publish    hand-off latency (last producer -> first consumer)
  max wk  max over WGs of (publish - input)
  crit    last publish of the phase - last publish of the phase before (its share of the launch span)
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

PHASES = ["T1 combine", "T2 wxo+x", "T3 ln2", "T4 fc1", "T5 fc2+x", "H0 ln1", "H1 qkv", "H2 self", "H3 wo+x",
          "H4 lnx", "H5 xq", "H6 q'"]
NPH = 12


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
    buf = torch.zeros((nl + 1) * 3 * NPH * 256, dtype=torch.int64, device="cuda")
    L.whisper_mi355x_set_pdec_stamps(C.c_void_p(buf.data_ptr()))
    st = ctx.create_state()
    V = L.whisper_n_vocab(ctx.ptr)
    forced = np.full((n_clips, n_tok), 50364, np.int32)  # the first timestamp token, every step
    rc, _ = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(c % 64) for c in range(n_clips)],
                                 n_tok, forced, [0], V)
    assert rc == 0, rc
    torch.cuda.synchronize()
    L.whisper_mi355x_set_pdec_stamps(None)
    s = buf.cpu().numpy().reshape(nl + 1, 3, NPH, 256).astype(np.float64) * 10.0  # ns
    if not s.any():
        print("no stamps (chain not taken?)")
        return 1
    s[s == 0] = np.nan
    t0 = np.nanmin(s)
    s -= t0
    tot = np.nanmax(s)
    print(f"{shape} {dtype} {n_clips} clips: step chain span {tot / 1e3:.1f} us over {nl + 1} launches")
    print(f"{'phase':12s} {'work us':>8s} {'max wk':>8s} {'operand':>8s} {'skew us':>8s} {'hand us':>8s} {'crit us':>8s}")
    mid = range(1, nl)
    sums = np.zeros(3)
    with np.errstate(all="ignore"):
        present = [p for p in range(NPH) if not np.all(np.isnan(s[mid.start:mid.stop, :2, p]))]
        for p in present:
            w = np.nanmean([np.nanmedian(s[k, 1, p] - s[k, 0, p]) for k in mid])
            wmax = np.nanmean([np.nanmax(s[k, 1, p] - s[k, 0, p]) for k in mid])
            pi = present.index(p)
            prev = [np.nanmax(s[k, 1, present[pi - 1]]) if pi > 0 else np.nanmin(s[k, 0, p]) for k in mid]
            crit = np.nanmean([np.nanmax(s[k, 1, p]) - prev[i] for i, k in enumerate(mid)])
            op = np.nanmean([np.nanmedian(s[k, 2, p] - s[k, 0, p]) for k in mid])
            sk = np.nanmean([np.nanmax(s[k, 1, p]) - np.nanmin(s[k, 1, p]) for k in mid])
            nx = present[pi + 1] if pi + 1 < len(present) else None
            h = np.nanmean([np.nanmin(s[k, 0, nx]) - np.nanmax(s[k, 1, p]) for k in mid]) if nx is not None else np.nan
            sums += (w, sk, 0 if np.isnan(h) else h)
            print(f"{PHASES[p]:12s} {w / 1e3:8.2f} {wmax / 1e3:8.2f} {op / 1e3:8.2f} {sk / 1e3:8.2f} {h / 1e3:8.2f} {crit / 1e3:8.2f}")
        gap = np.nanmean([np.nanmin(s[k + 1, 0, 0]) - np.nanmax(s[k, 1, NPH - 1]) for k in range(0, nl)])
        span = np.nanmean([np.nanmax(s[k, 1]) - np.nanmin(s[k, 0]) for k in mid])
    print(f"{'sum':12s} {sums[0] / 1e3:8.2f} {sums[1] / 1e3:8.2f} {sums[2] / 1e3:8.2f}")
    print(f"launch span (first input -> last publish) {span / 1e3:.2f} us; gap between launches {gap / 1e3:.2f} us")
    if os.environ.get("BDEC_STAMPS_DETAIL"):
        with np.errstate(all="ignore"):
            for p in range(NPH):
                wk = np.nanmean(np.stack([s[k, 1, p] - s[k, 0, p] for k in mid]), axis=0) / 1e3  # per WG, us
                if np.all(np.isnan(wk)):
                    continue
                by_xcd = [np.nanmean(wk[x::8]) for x in range(8)]
                worst = np.argsort(np.nan_to_num(wk, nan=-1))[::-1][:6]
                print(f"{PHASES[p]:12s} by XCD " + " ".join(f"{v:5.1f}" for v in by_xcd) +
                      "  slowest WGs " + " ".join(f"{w}:{wk[w]:.1f}" for w in worst))
    st.close()
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
