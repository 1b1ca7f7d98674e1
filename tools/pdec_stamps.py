"""Per-phase timeline of the persistent decode step (kernels/pdec.hip) from its debug clock stamps.

Every workgroup writes the 100 MHz clock when a phase's input arrived (its wait returned) and when it
published its output; the last captured step's stamps are summarised per phase over the layers:
  work    median over WGs of (publish - input)            the phase's own compute
  skew    max - min over WGs of the publish time          load imbalance / stragglers
  hand    min over WGs of the next input - max publish    hand-off latency (last producer -> first consumer)
usage: python tools/pdec_stamps.py [shape] [dtype] [clips] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]

PHASES = ["A ln+qkv", "B self", "C merge+o", "D ln+xq", "E cross", "F merge+xo", "G ln+fc1", "H fc2"]


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "large-v3+conf"
    dtype = sys.argv[2] if len(sys.argv) > 2 else "F16"
    n_clips = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    n_tok = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    from conftest import load_whisper_rs, model_path
    wrs = load_whisper_rs()
    from make_model import synthetic_pcm
    L = wrs.lib()
    ctx = wrs.WhisperContext(model_path(shape), dtype=getattr(wrs, dtype))
    nl = L.whisper_model_n_text_layer(ctx.ptr)
    buf = torch.zeros(256 * nl * 8 * 2, dtype=torch.int64, device="cuda")
    L.whisper_mi355x_set_pdec_stamps(C.c_void_p(buf.data_ptr()))
    st = ctx.create_state()
    V = L.whisper_n_vocab(ctx.ptr)
    forced = np.full((n_clips, n_tok), 50364, np.int32)  # the first timestamp token, every step
    rc, _ = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(c) for c in range(n_clips)], n_tok,
                                 forced, [0], V)
    assert rc == 0, rc
    torch.cuda.synchronize()
    L.whisper_mi355x_set_pdec_stamps(None)
    s = buf.cpu().numpy().reshape(256, nl, 8, 2).astype(np.float64) * 10.0  # ns (100 MHz clock)
    if not s.any():
        print("no stamps (persistent path not taken?)")
        return 1
    s[s == 0] = np.nan  # the attention phases stamp only the workgroups that hold a task
    t0 = np.nanmin(s[:, 0, 0, 0])
    s -= t0
    tot = np.nanmax(s[:, nl - 1, 7, 1])
    print(f"{shape} {dtype} {n_clips} clip(s): step {tot / 1e3:.1f} us over {nl} layers ({tot / nl / 1e3:.2f} us/layer)")
    print(f"{'phase':12s} {'work us':>8s} {'skew us':>8s} {'hand us':>8s} {'first-in':>9s} {'last-sig':>9s}")
    sums = np.zeros(3)
    for p in range(8):
        work = np.nanmedian(s[:, :, p, 1] - s[:, :, p, 0], axis=0)
        skew = np.nanmax(s[:, :, p, 1], axis=0) - np.nanmin(s[:, :, p, 1], axis=0)
        if p < 7:
            nxt = s[:, :, p + 1, 0]
        else:
            nxt = np.concatenate([s[:, 1:, 0, 0], np.full((256, 1), np.nan)], axis=1)
        with np.errstate(all="ignore"):
            hand = np.nanmin(nxt, axis=0) - np.nanmax(s[:, :, p, 1], axis=0)
        w, k, h = np.nanmean(work) / 1e3, np.nanmean(skew) / 1e3, np.nanmean(hand) / 1e3
        sums += (w, k, h)
        print(f"{PHASES[p]:12s} {w:8.2f} {k:8.2f} {h:8.2f} {np.nanmin(s[:, 1, p, 0]) / 1e3:9.2f} {np.nanmax(s[:, 1, p, 1]) / 1e3:9.2f}")
    print(f"{'sum':12s} {sums[0]:8.2f} {sums[1]:8.2f} {sums[2]:8.2f}   (layer 1 absolute times in the last columns)")
    st.close()
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
