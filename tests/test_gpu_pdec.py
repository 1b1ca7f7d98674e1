"""The persistent decode step (nobs-whisper_amd/csrc/kernels/pdec.hip): every decoder layer of a decode
step of <= 4 clips (the app's one clip per call, whisper.rs:83-85 / state.rs:147) in ONE launch, the
cross K/V cache form.

  * whisper_full f16 through it: token ids, timestamps, text and per-window decisions identical to the
    oracle on every model width the kernel is built for (d 384 / 512 / 768 / 1280; 1024 is in
    tests/test_gpu_fulldepth.py), with the reference's FullParams, prompted and auto-language cases
    (a clip with an oracle near tie <= F16_GAP nats: identical up to that step);
  * GGML-block files (the app's catalog: small-q5_1, medium-q5_0, large-v3-q5_0; plus q4_1 / q8_0), both
    through the block-streaming kernel (f16 compute) and the default expanded copy: exact against the
    oracle like the f16 cases;
  * a batch of 4 clips (the largest it takes) against the oracle clip by clip;
  * the give-up path: with a zero spin limit every launch gives up and the step is re-run on the
    per-kernel path: results equal the per-kernel path's (WHISPER_MI355X_PDEC=0) bit for bit, and the
    state's give-up counter says so (every other case asserts it is 0);
  * batch == single on the default path (3 clips of different lengths: persistent steps at 3, 2, 1 clips);
  * two states on two host threads (persistent steps serialised by the engine): each equals its
    single-threaded run.
Each case checks that the persistent kernel actually ran (its kernel-timing class counted launches).
"""
import threading

import pytest

from make_model import synthetic_pcm
from margin_gate import assert_closed_before_divergence, assert_diverges_only_at_close_calls, kept_token_margins
from oracle_py import cached_full, reference_params

pytestmark = pytest.mark.gpu

K_PDEC = 7
# f16 is compared exactly on clips whose every greedy step the oracle decided by more than F16_GAP nats
# (f16 teacher-forced logits sit within ~0.015 of the oracle's, tests/test_gpu_fulldepth.py); where the
# oracle itself has a near tie, exactly up to that step (the round-2 rule)
F16_GAP = 0.05


def oracle_full(shape, clip, lang="en", prompt=None, t_inc=0.2):
    from conftest import model_path
    rp = reference_params(lang, prompt=prompt)
    rp.temperature_inc = t_inc
    return cached_full(model_path(shape), ("clip", clip), lambda: synthetic_pcm(clip), rp)


def ints(segs):
    return [([t[0] for t in s.tokens], s.t0, s.t1) for s in segs]


def ref_ints(ref):
    return [(s["tokens"], s["t0"], s["t1"]) for s in ref["segments"]]


DEC_KEYS = ("seek", "temp_idx", "failed0", "logprob_fail0", "result_len0", "no_speech")


def pdec_launches(wrs, st):
    import ctypes as C
    out = (C.c_double * 3)()
    assert wrs.lib().whisper_mi355x_kernel_stats(st.ptr, K_PDEC, out) == 0
    return int(out[1])


# the reference's FullParams (temperature_inc 0.2) where the oracle decides every window at t = 0 (the
# cases of tests/test_gpu_configs.py F16_CASES), greedy-only (0.0) for small-4L
CASES = [("tiny.en+conf", 0, "en", "DEFAULT", 0.2), ("tiny.en+conf", 1, None, None, 0.2), ("base+conf", 0, "en", None, 0.2),
         ("base+conf", 1, "en", "DEFAULT", 0.2), ("small-4L+conf", 0, "en", None, 0.0),
         ("large-v3-2L+conf", 0, "en", None, 0.2), ("large-v3-2L+conf", 1, None, None, 0.2),
         ("large-v3-2L+conf", 0, None, "DEFAULT", 0.2)]


@pytest.mark.parametrize("shape,clip,lang,prompt,t_inc", CASES)
def test_pdec_full_f16_exact(wrs, monkeypatch, shape, clip, lang, prompt, t_inc):
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    prompt = wrs.DEFAULT_VOCABULARY if prompt == "DEFAULT" else prompt
    ref = oracle_full(shape, clip, lang, prompt, t_inc)
    assert all(d["temp_idx"] == 0 for d in ref["decisions"]), ref["decisions"]
    ctx = wrs.WhisperContext(model_path(shape), dtype=wrs.F16)
    st = ctx.create_state()
    wrs.lib().whisper_mi355x_kernel_timing(st.ptr, 1 << K_PDEC)
    gp = wrs.reference_full_params(lang, initial_prompt=prompt)
    gp.temperature_inc = t_inc
    assert st.full(gp, synthetic_pcm(clip)) == 0
    n = pdec_launches(wrs, st)
    gave_up = st.pdec_give_ups()
    segs, dec = st.segments(), st.decisions()
    st.close()
    ctx.close()
    assert n > 0, "the persistent decode step did not run"
    assert gave_up == 0, f"{gave_up} persistent launches gave up (re-run on the per-kernel path)"
    exp, margins = kept_token_margins(ref)
    if min(margins) > F16_GAP:
        assert ints(segs) == ref_ints(ref)
        assert [s.text for s in segs] == [s["text"] for s in ref["segments"]]
        assert [tuple(d[k] for k in DEC_KEYS) for d in dec] == [tuple(d[k] for k in DEC_KEYS) for d in ref["decisions"]]
        print(f"{shape} clip {clip}: {n} persistent steps, {len(exp)} tokens identical")
    else:  # the oracle decided a step by <= F16_GAP nats: exact up to the first such near tie
        got = [t for sg in ints(segs) for t in sg[0]]
        k = assert_diverges_only_at_close_calls(got, exp, margins, F16_GAP, 4)
        ns, nw = assert_closed_before_divergence(segs, dec, ref, k)
        print(f"{shape} clip {clip}: {n} persistent steps, {k} of {len(exp)} tokens identical "
              f"(oracle near tie {min(margins):.4f} nats); {ns} segment(s), {nw} window decision(s) before it identical")


QUANT_CASES = [("small-4L+conf+q5_1", 1, "en", None, 0.2), ("large-v3-2L+conf+q5_0", 0, "en", None, 0.2),
               ("large-v3-turbo-2L+conf+q4_1", 1, "en", None, 0.2), ("large-v3-2L+conf+q8_0", 1, None, None, 0.2)]


@pytest.mark.parametrize("blocks", [1, 0])
@pytest.mark.parametrize("shape,clip,lang,prompt,t_inc", QUANT_CASES)
def test_pdec_quant_f16_exact(wrs, monkeypatch, shape, clip, lang, prompt, t_inc, blocks):
    """blocks 1: the persistent kernel streams the GGML blocks (dequantized in registers); 0 (the
    default): it reads the context's expanded compute-type copy of the same weights."""
    wrs.lib().whisper_mi355x_set_pdec_blocks(blocks)
    try:
        test_pdec_full_f16_exact(wrs, monkeypatch, shape, clip, lang, prompt, t_inc)
    finally:
        wrs.lib().whisper_mi355x_set_pdec_blocks(0)


def test_pdec_batch4_vs_oracle(wrs, monkeypatch):
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    shape = "base+conf"
    ctx = wrs.WhisperContext(model_path(shape), dtype=wrs.F16)
    st = ctx.create_state()
    wrs.lib().whisper_mi355x_kernel_timing(st.ptr, 1 << K_PDEC)
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    assert st.full_batch(p, [synthetic_pcm(k) for k in range(4)]) == 0
    assert pdec_launches(wrs, st) > 0
    for j in range(4):
        ref = oracle_full(shape, j, "en", None, t_inc=0.0)
        assert ints(st.batch_segments(j)) == ref_ints(ref), j
    st.close()
    ctx.close()


def _run(wrs, path, clips, dtype):
    ctx = wrs.WhisperContext(path, dtype=dtype)
    st = ctx.create_state()
    wrs.lib().whisper_mi355x_kernel_timing(st.ptr, 1 << K_PDEC)
    assert st.full_batch(wrs.reference_full_params("en"), clips) == 0
    out = [ints(st.batch_segments(j)) for j in range(len(clips))], [st.decisions(j) for j in range(len(clips))]
    n = (pdec_launches(wrs, st), st.pdec_give_ups())
    st.close()
    ctx.close()
    return out, n


@pytest.mark.parametrize("dtype", ["F16", "BF16"])
def test_pdec_give_up_reruns_step(wrs, monkeypatch, capfd, dtype):
    """Zero spin limit: every persistent launch gives up at its first wait; the engine re-runs each
    step on the per-kernel path, so the results are those of WHISPER_MI355X_PDEC=0 exactly."""
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    monkeypatch.setenv("WHISPER_MI355X_STATE_POOL", "0")
    path = model_path("tiny+conf")
    clips = [synthetic_pcm(k) for k in range(2)]
    L = wrs.lib()
    monkeypatch.setenv("WHISPER_MI355X_PDEC", "0")
    plain, n0 = _run(wrs, path, clips, getattr(wrs, dtype))
    assert n0 == (0, 0)
    monkeypatch.delenv("WHISPER_MI355X_PDEC")
    L.whisper_mi355x_set_pdec_spin(0)
    try:
        forced, n1 = _run(wrs, path, clips, getattr(wrs, dtype))
    finally:
        L.whisper_mi355x_set_pdec_spin(5000000)
    # the first launch gives up and is re-run; the state's next steps then take the per-kernel path for
    # the backoff period instead of timing out again (kernel stats count the give-ups)
    assert n1[0] > 0 and n1[1] >= 1, n1
    assert forced == plain


def test_pdec_two_threads(wrs, monkeypatch):
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    path = model_path("base+conf")
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    clips = [synthetic_pcm(k) for k in range(2)]
    p = wrs.reference_full_params("en")
    single = []
    for c in clips:
        st = ctx.create_state()
        assert st.full(p, c) == 0
        single.append(ints(st.segments()))
        st.close()
    res = [None, None]

    def work(i):
        st = ctx.create_state()
        rc = st.full(p, clips[i])
        res[i] = (rc, ints(st.segments()))
        st.close()
    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    ctx.close()
    assert [r[0] for r in res] == [0, 0]
    assert [r[1] for r in res] == single


@pytest.mark.parametrize("shape", ["base+conf", "large-v3-2L+conf"])
def test_pdec_batch_equals_single(wrs, monkeypatch, shape):
    """The default path (no switches): a batch of 3 clips of different lengths, whose decode steps run the
    persistent kernel at 3, 2 and 1 active clips as clips finish, equals each clip run alone (1 clip per
    step) bit for bit: token ids, probabilities, timestamps, text and window decisions (the
    key-split count and the LayerNorm order no longer depend on the clip count). large-v3-2L (20 heads)
    deals 2-3 cross-attention tasks to some workgroups at 2-3 clips; base (8 heads) one each."""
    from conftest import model_path
    monkeypatch.setenv("WHISPER_MI355X_CROSS", "cache")
    path = model_path(shape)
    clips = [synthetic_pcm(k, seconds=30.0 - 4.0 * k) for k in range(3)]
    p = wrs.reference_full_params("en")
    p.temperature_inc = 0.0
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)

    def run(batch):
        st = ctx.create_state()
        wrs.lib().whisper_mi355x_kernel_timing(st.ptr, 1 << K_PDEC)
        assert st.full_batch(p, batch) == 0
        out = [([tuple(t) for t in s.tokens], s.t0, s.t1, s.text) for j in range(len(batch)) for s in st.batch_segments(j)], \
            [st.decisions(j) for j in range(len(batch))]
        n, g = pdec_launches(wrs, st), st.pdec_give_ups()
        st.close()
        assert n > 0 and g == 0, (n, g)
        return out
    together = run(clips)
    alone = [run([c]) for c in clips]
    ctx.close()
    assert together[0] == [seg for a in alone for seg in a[0]]
    assert together[1] == [a[1][0] for a in alone]
