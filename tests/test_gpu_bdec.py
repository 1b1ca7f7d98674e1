"""The batched persistent decoder chain (nobs-whisper_amd/csrc/kernels/bdec.hip): decode steps of 5..128 clips
in the direct cross form, one chain launch per layer around the pass over the encoder output (the headline's
128-clip batch, BASELINE configs[3], and its 16-clip shard at 8 GPUs; whisper.rs:127-129 batched).

  * teacher-forced logits against the oracle along its fixed-work greedy sequences, at clip counts that
    exercise every row-group layout (5: one partial group; 40: two groups, the second with 8 rows; 128:
    four full groups): f16 max |dlogit| / max |logit| <= 1e-3 at every step (the north star's bound),
    bf16 max |dlogit| <= 0.5 (tests/test_gpu_fulldepth.py's bars);
  * the chain against the launch chain it replaces (WHISPER_MI355X_BDEC=0) on the same batch: the same
    greedy tokens wherever neither run met an oracle near tie (f16), so a regression shows up on clips
    whose decisions are confident;
  * whisper_full (real termination, the reference's FullParams, greedy attempt) at 40 clips: token ids,
    timestamps and text of every spot clip identical to the oracle up to its first near tie;
  * the kernel class of the chain (8) counted launches, and no launch gave up.
"""
import ctypes as C

import numpy as np
import pytest

from make_model import synthetic_pcm
from margin_gate import assert_closed_before_divergence, assert_diverges_only_at_close_calls, kept_token_margins
from oracle_py import cached_full, reference_params

pytestmark = pytest.mark.gpu

K_BDEC = 8
N_TOK = 24
F16_REL_TOL = 1e-3
BF16_TOL = 0.5
F16_GAP = 0.05
SHAPE = "large-v3-2L+conf"


def _fixed_ref(path, clip):
    return cached_full(path, ("clip", clip), lambda: synthetic_pcm(clip), reference_params("en", fixed_tokens=N_TOK))


def _forced_run(wrs, path, dtype, n, spot, monkeypatch, bdec=True):
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "direct")
    monkeypatch.setenv("WHISPER_MI355X_BDEC", "1" if bdec else "0")
    refs = [_fixed_ref(path, c % 64) for c in spot]
    forced = np.array([refs[0]["step_tokens"]] * n, np.int32)
    for k, c in enumerate(spot):
        forced[c] = refs[k]["step_tokens"]
    ctx = wrs.WhisperContext(path, dtype=getattr(wrs, dtype))
    st = ctx.create_state()
    L = wrs.lib()
    L.whisper_mi355x_kernel_timing(st.ptr, 1 << K_BDEC)
    V = L.whisper_n_vocab(ctx.ptr)
    rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(k % 64) for k in range(n)], N_TOK,
                                  forced, list(spot), V)
    assert rc == 0, rc
    out = (C.c_double * 3)()
    L.whisper_mi355x_kernel_stats(st.ptr, K_BDEC, out)
    assert st.info()["direct"]
    assert st.pdec_give_ups() == 0
    st.close()
    ctx.close()
    return lg, refs, int(out[1])


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
@pytest.mark.parametrize("n", [5, 40, 128])
def test_bdec_teacher_forced_vs_oracle(wrs, monkeypatch, n, dtype):
    from conftest import model_path
    path = model_path(SHAPE)
    spot = (0, n - 1) if n > 1 else (0,)
    lg, refs, launches = _forced_run(wrs, path, dtype, n, spot, monkeypatch)
    assert launches >= (N_TOK - 1) * 3, launches  # L + 1 chain launches per decode step
    for k, c in enumerate(spot):
        ref = refs[k]["step_logits"].astype(np.float64)
        got = lg[:, k, :].astype(np.float64)
        assert np.isfinite(got).all()
        per_step = np.abs(got - ref).max(axis=1)
        rel = per_step / np.abs(ref).max(axis=1)
        print(f"bdec {dtype} n={n} clip {c}: worst |dlogit| {per_step.max():.4f}, relative {rel.max():.2e}")
        if dtype == "F16":
            assert rel.max() <= F16_REL_TOL, (rel.max(), int(rel.argmax()))
        else:
            assert per_step.max() <= BF16_TOL, (per_step.max(), int(per_step.argmax()))


def test_bdec_matches_launch_chain(wrs, monkeypatch):
    """f16, 40 clips, fixed work (forced tokens): the chain's logits against the launch chain's, both against
    the oracle; the chain may not be further from the oracle than the launch chain by more than the bar."""
    from conftest import model_path
    path = model_path(SHAPE)
    spot = (0, 17, 39)
    a, refs, na = _forced_run(wrs, path, "F16", 40, spot, monkeypatch, bdec=True)
    b, _, nb = _forced_run(wrs, path, "F16", 40, spot, monkeypatch, bdec=False)
    assert na > 0 and nb == 0
    for k, c in enumerate(spot):
        ref = refs[k]["step_logits"].astype(np.float64)
        da = np.abs(a[:, k, :] - ref).max()
        db = np.abs(b[:, k, :] - ref).max()
        dab = np.abs(a[:, k, :].astype(np.float64) - b[:, k, :]).max()
        print(f"clip {c}: chain vs oracle {da:.4f}, launch chain vs oracle {db:.4f}, chain vs launch chain {dab:.4f}")
        assert dab <= 2 * F16_REL_TOL * np.abs(ref).max(), dab


def test_bdec_whisper_full_vs_oracle(wrs, monkeypatch):
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "direct")
    monkeypatch.setenv("WHISPER_MI355X_BDEC", "1")
    path = model_path(SHAPE)
    n = 40
    clips = [synthetic_pcm(k % 64) for k in range(n)]
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    st = ctx.create_state()
    wrs.lib().whisper_mi355x_kernel_timing(st.ptr, 1 << K_BDEC)
    assert st.full_batch(p, clips) == 0
    out = (C.c_double * 3)()
    wrs.lib().whisper_mi355x_kernel_stats(st.ptr, K_BDEC, out)
    assert out[1] > 0, "the chain did not run"
    for j in (0, 13, 26, 39):
        rp = reference_params("en")
        rp.temperature_inc = 0.0
        ref = cached_full(path, ("clip", j % 64), lambda s=j % 64: synthetic_pcm(s), rp)
        segs, dec = st.batch_segments(j), st.decisions(j)
        exp, margins = kept_token_margins(ref)
        got = [t[0] for s in segs for t in s.tokens]
        if min(margins) > F16_GAP:
            assert [([t[0] for t in s.tokens], s.t0, s.t1) for s in segs] == [(s["tokens"], s["t0"], s["t1"]) for s in ref["segments"]], j
            assert [s.text for s in segs] == [s["text"] for s in ref["segments"]], j
        else:
            k = assert_diverges_only_at_close_calls(got, exp, margins, F16_GAP, 4)
            assert_closed_before_divergence(segs, dec, ref, k)
    st.close()
    ctx.close()
