"""Parity at the BASELINE models' real depth (VERDICT r3 "next" #1).

The other config tests run the BASELINE shapes at reduced depth (tools/make_model.py SHAPES, e.g.
large-v3-2L) so the CPU oracle stays fast. Here the oracle runs the full stacks:
  large-v3       (src-tauri/src/model.rs:98-107)   128 mels, d 1280, 20 heads, 32 + 32 layers
  large-v3-turbo (model.rs:108-117)                 large-v3 dims, 32 + 4 layers
  medium         (model.rs medium / medium-q5_0)    80 mels, d 1024, 16 heads, 24 + 24 layers
all with the "+conf" decoders (make_model.CONF_SCALE) so windows end the way a trained model's do.

(a) f16 whisper_full (the reference's FullParams, whisper.rs:88-124, greedy attempt only:
    temperature_inc 0) on two clips per shape, in both cross-attention forms: token ids,
    timestamps, segment text and per-window decisions identical to the oracle, up to the first oracle
    near tie (F16_GAP, the rule of every f16 whisper_full test): large-v3-turbo clip 1 has a step the
    oracle decides by 0.0049 nats, where the persistent step (cache form, 1 clip) took the other token.
(b) BASELINE configs[3]'s own workload (bench.py's step): large-v3 at 128 clips in one batch, the
    direct cross form with the bench's split count, fixed-work mode (128 tokens per clip, EOT
    suppressed), every clip teacher-forced along the oracle's greedy sequence of a spot clip
    (whisper_mi355x_full_batch_forced: the same kernels and graphs as the bench). For 4 spot clips
    the raw logits of all 128 steps are compared with the oracle's along the same sequence:
      f16  : max_v |dlogit| / max_v |logit_oracle| <= 1e-3 at every step (the north star's bound);
      bf16 : max_v |dlogit| <= BF16_DEEP_TOL at every step, and the argmax agrees wherever the
             oracle's top-2 gap exceeds BF16_FLIP_GAP.
    BF16_DEEP_TOL = 0.5 (round 5; round 4 had 2.0, fixed before its first run, and measured a worst step
    of 0.236, profiles/r04_gputests_fulldepth_v5.txt): a 2x regression of the headline dtype's decoder
    now fails; the measured worst step is printed. BF16_FLIP_GAP = 0.25 (round 6, VERDICT r5 weak 3: the
    largest gap of a measured bf16 flip was 0.083; the old rule, 2 * tol = 1.0 nats, could not fail).
(c) BASELINE configs[4]'s own workload: large-v3-turbo (32 + 4) with fp8 weights (e4m3 encoder
    GEMMs, bf16 decoder) at 256 clips in one call (two concurrent 128-clip halves, direct cross form),
    fixed work, teacher-forced like (b); 4 spot clips spread over both halves against the f16-numerics
    oracle: max_v |dlogit| <= FP8_DEEP_TOL at every step, and the argmax agrees wherever the oracle's
    top-2 gap exceeds FP8_FLIP_GAP. Round 6 set both from round 5's measurements instead
    of the bars fixed before the first run (4.0 nats, and flips allowed up to 8 nats, which could not fail):
    FP8_DEEP_TOL 2.5 (measured worst 1.61), FP8_FLIP_GAP 1.0 (measured flips at gaps up to 0.54).
(d) The two BASELINE workloads round 5 left without a full-depth comparison (VERDICT r5 missing 2):
    small (12 + 12 layers, model.rs:76-86) in bf16 at 32 clips, configs[2], on the bench's default path for that
    batch (the cross K/V cache form, the split-K launch chain); and large-v3 at 16 clips, one rank's shard of
    configs[3] at 8 GPUs (the cache-form launch chain), f16 and bf16. Teacher-forced like (b), same bars.
Near ties in (a) (VERDICT r4 "next" #1): the identical token prefix must reach the tie, and every segment
that closes before it (tokens, t0, t1, text) and every window that ends before it (its decisions) must
equal the oracle's (margin_gate.assert_closed_before_divergence).
The oracle is the slow side (~13 s per large-v3 encoder pass on 16 threads): each spot clip is its own
test so no single test runs for minutes; oracle results (and their raw per-step logits, recorded by the
oracle's fixed-work mode instead of a second teacher-forced pass) are computed once per session
(oracle_py.cached_full, shared with the other modules).
"""
import numpy as np
import pytest

from make_model import synthetic_pcm
from margin_gate import assert_closed_before_divergence, assert_diverges_only_at_close_calls, kept_token_margins
from oracle_py import cached_full, reference_params

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

F16_REL_TOL = 1e-3
BF16_DEEP_TOL = 0.5
BF16_FLIP_GAP = 0.25
FP8_DEEP_TOL = 2.5
FP8_FLIP_GAP = 1.0
F16_FLIP_GAP = 0.05  # f16 teacher-forced logits sit within ~0.015 of the oracle's (the F16_GAP rule below)
# (a): exact where the oracle decided every greedy step by more than F16_GAP nats, else exact up to the
# first such near tie: the rule of every f16 whisper_full test (tests/test_gpu_pdec.py);
# f16 teacher-forced logits sit within ~0.015 of the oracle's
F16_GAP = 0.05
N_TOK = 128
N_CLIPS = 128
SPOT = (0, 41, 86, 127)



def _ints(segs):
    return [([t[0] for t in s.tokens], s.t0, s.t1) for s in segs]


# ---- (a) f16 whisper_full, token-exact -----------------------------------------------------------------
FULL_CASES = [("large-v3+conf", 0), ("large-v3+conf", 1), ("large-v3-turbo+conf", 0), ("large-v3-turbo+conf", 1),
              ("medium+conf", 0), ("medium+conf", 1)]


@pytest.mark.parametrize("cross", ["direct", "cache"])
@pytest.mark.parametrize("shape,clip", FULL_CASES)
def test_full_depth_f16_exact(wrs, monkeypatch, shape, clip, cross):
    from conftest import model_path
    pcm = synthetic_pcm(clip)
    rp = reference_params("en")
    rp.temperature_inc = 0.0
    ref = cached_full(model_path(shape), ("clip", clip), lambda: pcm, rp)  # a fresh oracle state per call
    monkeypatch.setenv("WHISPER_MI355X_CROSS", cross)
    ctx = wrs.WhisperContext(model_path(shape), dtype=wrs.F16)
    st = ctx.create_state()
    gp = wrs.reference_full_params("en")
    gp.temperature_inc = 0.0
    assert st.full(gp, pcm) == 0
    assert st.info()["direct"] == (cross == "direct")
    segs, dec = st.segments(), st.decisions()
    st.close()
    ctx.close()
    exp = [(s["tokens"], s["t0"], s["t1"]) for s in ref["segments"]]
    kept, margins = kept_token_margins(ref)
    if min(margins) > F16_GAP:
        assert _ints(segs) == exp
        assert [s.text for s in segs] == [s["text"] for s in ref["segments"]]
        keys = ("seek", "temp_idx", "failed0", "logprob_fail0", "result_len0", "no_speech")
        assert [tuple(d[k] for k in keys) for d in dec] == [tuple(d[k] for k in keys) for d in ref["decisions"]]
        print(f"{shape} clip {clip} {cross}: {sum(len(s['tokens']) for s in ref['segments'])} tokens identical "
              f"over {len(ref['decisions'])} window(s)")
    else:  # the oracle decided a step by <= F16_GAP nats: exact up to the first such near tie
        got = [t for sg in _ints(segs) for t in sg[0]]
        k = assert_diverges_only_at_close_calls(got, kept, margins, F16_GAP, 4)
        ns, nw = assert_closed_before_divergence(segs, dec, ref, k)
        print(f"{shape} clip {clip} {cross}: {k} of {len(kept)} tokens identical (oracle near tie {min(margins):.4f} nats); "
              f"{ns} segment(s) and {nw} window decision(s) before it identical")


# ---- (b) large-v3, 128 clips, direct form, fixed work, teacher-forced -----------------------------------
_GPU_LG = {}    # (shape, dtype, clips) -> GPU logits [N_TOK][len(spot)][V]


def _oracle_fixed(shape, clip):
    """The oracle's greedy fixed-work run of a clip (N_TOK step tokens) and the raw logits of every step
    along it (the teacher-forced reference)."""
    from conftest import model_path
    ref = cached_full(model_path(shape), ("clip", clip), lambda: synthetic_pcm(clip),
                      reference_params("en", fixed_tokens=N_TOK))
    assert len(ref["step_tokens"]) == N_TOK and ref["step_logits"].shape[0] == N_TOK, \
        (len(ref["step_tokens"]), ref["step_logits"].shape)
    return ref


def _oracle_seq(clip, shape="large-v3+conf"):
    return _oracle_fixed(shape, clip)["step_tokens"]


def _oracle_logits(clip, shape="large-v3+conf"):
    return _oracle_fixed(shape, clip)["step_logits"].astype(np.float64)


def _gpu_logits(wrs, dtype, shape="large-v3+conf", n_clips=N_CLIPS, spot=SPOT, seeds=None, direct=True):
    """Teacher-forced raw logits [N_TOK][len(spot)][V] of the spot positions of one n_clips call. Position j holds
    synthetic_pcm(seeds[j]) (default j % 128); the spot positions decode the oracle sequence of their own seed,
    the others that of a spot clip. direct: the cross form the call must have taken (the default per-call
    choice: direct above 32 clips, the cache form up to 32)."""
    from conftest import model_path
    seeds = list(seeds) if seeds is not None else [j % 128 for j in range(n_clips)]
    key = (shape, dtype, n_clips, spot, tuple(seeds))
    if key not in _GPU_LG:
        seqs = [_oracle_seq(seeds[c], shape) for c in spot]
        forced = np.array([seqs[j % len(spot)] for j in range(n_clips)], np.int32)
        # the spot clips decode their own oracle sequence
        for k, c in enumerate(spot):
            forced[c] = seqs[k]
        clips = [synthetic_pcm(s) for s in seeds]
        ctx = wrs.WhisperContext(model_path(shape), dtype=getattr(wrs, dtype))
        st = ctx.create_state()
        V = wrs.lib().whisper_n_vocab(ctx.ptr)
        rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), clips, N_TOK, forced, list(spot), V)
        assert rc == 0, rc
        assert st.info()["direct"] == direct, st.info()
        assert st.pdec_give_ups() == 0
        st.close()
        ctx.close()
        _GPU_LG[key] = lg
    return _GPU_LG[key]


def _check(dtype, clip, got, ref, label, model="large-v3"):
    assert np.isfinite(got).all()
    d = np.abs(got.astype(np.float64) - ref)
    per_step = d.max(axis=1)
    scale = np.abs(ref).max(axis=1)
    rel = per_step / scale
    top2 = np.sort(ref, axis=1)[:, -2:]
    gap = top2[:, 1] - top2[:, 0]
    flips = [(i, float(gap[i])) for i in range(N_TOK) if int(np.argmax(got[i])) != int(np.argmax(ref[i]))]
    print(f"{model} {dtype} {label} clip {clip}: worst step |dlogit| {per_step.max():.4f} (step {int(per_step.argmax())}), "
          f"relative {rel.max():.2e}, median relative {np.median(rel):.2e}, logit scale {scale.mean():.1f}, "
          f"argmax flips {flips}")
    if dtype == "F16":
        assert rel.max() <= F16_REL_TOL, (rel.max(), int(rel.argmax()))
        assert all(g <= F16_FLIP_GAP for _, g in flips), flips
    else:
        tol, gap_bar = (FP8_DEEP_TOL, FP8_FLIP_GAP) if dtype == "FP8_ENC" else (BF16_DEEP_TOL, BF16_FLIP_GAP)
        assert per_step.max() <= tol, (per_step.max(), int(per_step.argmax()))
        assert all(g <= gap_bar for _, g in flips), flips


_FEW_LG = {}


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
@pytest.mark.parametrize("n_clips", [1, 4])
def test_largev3_few_clips_teacher_forced(wrs, monkeypatch, dtype, n_clips):
    """The app's pattern at full depth: 1 (and 4) clips, the cross K/V cache form, every step one
    persistent launch (kernels/pdec.hip; its kernel class counts the launches), teacher-forced along the
    oracle's fixed-work sequences of the spot clips: the same bars as the 128-clip case."""
    from conftest import model_path
    monkeypatch.delenv("WHISPER_MI355X_CROSS", raising=False)
    spot = SPOT[:n_clips]
    key = (dtype, n_clips)
    if key not in _FEW_LG:
        seqs = np.array([_oracle_seq(c) for c in spot], np.int32)
        ctx = wrs.WhisperContext(model_path("large-v3+conf"), dtype=getattr(wrs, dtype))
        st = ctx.create_state()
        L = wrs.lib()
        L.whisper_mi355x_kernel_timing(st.ptr, 1 << 7)
        V = L.whisper_n_vocab(ctx.ptr)
        rc, lg = st.full_batch_forced(wrs.reference_full_params("en"), [synthetic_pcm(c) for c in spot], N_TOK, seqs,
                                      list(range(n_clips)), V)
        assert rc == 0, rc
        import ctypes as C
        out = (C.c_double * 3)()
        L.whisper_mi355x_kernel_stats(st.ptr, 7, out)
        assert not st.info()["direct"] and out[1] >= N_TOK - 1, (st.info(), out[1])
        assert st.pdec_give_ups() == 0
        st.close()
        ctx.close()
        _FEW_LG[key] = lg
    for k, c in enumerate(spot):
        _check(dtype, c, _FEW_LG[key][:, k, :], _oracle_logits(c), f"persistent b{n_clips}")


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
@pytest.mark.parametrize("k", range(len(SPOT)))
def test_largev3_b128_teacher_forced(wrs, monkeypatch, dtype, k):
    monkeypatch.delenv("WHISPER_MI355X_CROSS", raising=False)
    clip = SPOT[k]
    ref = _oracle_logits(clip)
    _check(dtype, clip, _gpu_logits(wrs, dtype)[:, k, :], ref, "b128")


# ---- (c) large-v3-turbo fp8 weights, 256 clips (BASELINE configs[4]), teacher-forced ------------------------
TURBO_SPOT = (0, 77, 170, 255)  # two spot clips in each 128-clip half


@pytest.mark.parametrize("k", range(len(TURBO_SPOT)))
def test_turbo_fp8_b256_teacher_forced(wrs, monkeypatch, k):
    monkeypatch.delenv("WHISPER_MI355X_CROSS", raising=False)
    clip = TURBO_SPOT[k]
    ref = _oracle_logits(clip % 128, "large-v3-turbo+conf")
    got = _gpu_logits(wrs, "FP8_ENC", "large-v3-turbo+conf", 256, TURBO_SPOT)[:, k, :]
    _check("FP8_ENC", clip, got, ref, "b256", "large-v3-turbo")



# ---- (d) configs[2] (small bf16, 32 clips) and configs[3]'s 8-GPU shard (large-v3, 16 clips), full depth -----
SMALL_SPOT = (0, 9, 20, 31)


@pytest.mark.parametrize("k", range(len(SMALL_SPOT)))
def test_small_b32_bf16_teacher_forced(wrs, monkeypatch, k):
    """BASELINE configs[2]: small (12 + 12) bf16, 32 clips in one call, the bench's default path for that batch
    (cross K/V cache form, split-K launch chain: no persistent step above 4 clips)."""
    monkeypatch.delenv("WHISPER_MI355X_CROSS", raising=False)
    clip = SMALL_SPOT[k]
    ref = _oracle_logits(clip, "small+conf")
    got = _gpu_logits(wrs, "BF16", "small+conf", 32, SMALL_SPOT, direct=False)[:, k, :]
    _check("BF16", clip, got, ref, "b32", "small")


SHARD_SEEDS = [0, 41, 86, 127] + list(range(1, 13))  # the (b) spot clips (their oracle runs are shared) + 12 more
SHARD_SPOT = (0, 1, 2, 3)


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
@pytest.mark.parametrize("k", range(len(SHARD_SPOT)))
def test_largev3_b16_shard_teacher_forced(wrs, monkeypatch, dtype, k):
    """One rank's shard of configs[3] at 8 GPUs (128 clips / 8 = 16 per rank): large-v3 at 16 clips, the cross
    K/V cache form and its launch chain, teacher-forced along the oracle sequences of the (b) spot clips."""
    monkeypatch.delenv("WHISPER_MI355X_CROSS", raising=False)
    seed = SHARD_SEEDS[SHARD_SPOT[k]]
    ref = _oracle_logits(seed)
    got = _gpu_logits(wrs, dtype, "large-v3+conf", 16, SHARD_SPOT, seeds=SHARD_SEEDS, direct=False)[:, k, :]
    _check(dtype, seed, got, ref, "b16 shard")
