"""The reference's boundary caller end to end: the C++ WhisperEngine mirror (host/whisper_engine.cpp,
a line-by-line restatement of src-tauri/src/whisper.rs) over the HIP engine, against the same caller
logic applied to the CPU oracle's whisper_full (not against the engine itself):

  expected = filter_hallucinations(trim(concat(to_str_lossy(segment_i))))     whisper.rs:131-144

on a fresh oracle state per call (whisper.rs:83-85), for every initial-prompt branch
(whisper.rs:98-105), for transcribe_chunked's context chaining (whisper.rs:152-197), and for two
states of one context transcribing concurrently from two threads (Arc<WhisperEngine> shared by the
worker and stop threads, state.rs:116, 686). The clips are ones whose oracle windows are all decided
at t = 0 with the reference's FullParams (asserted), so every integer decision is comparable.
"""
import threading

import pytest

from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params

pytestmark = pytest.mark.gpu

SHAPE = "base+conf"
CTX = "Hello world thank you"


def expected_text(wrs, o, pcm, language, prompt):
    o.new_state()
    res = o.full(pcm, reference_params(language, prompt=prompt))
    assert res["rc"] == 0
    assert all(d["temp_idx"] == 0 for d in res["decisions"]), res["decisions"]
    joined = "".join(s["text"].decode("utf-8", "replace") for s in res["segments"])
    return wrs.filter_hallucinations(joined.strip())


@pytest.fixture(scope="module")
def oracle():
    from conftest import model_path
    o = Oracle(model_path(SHAPE), mode=1, n_threads=16)
    yield o
    o.close()


@pytest.fixture(scope="module")
def engine(wrs):
    from conftest import model_path
    e = wrs.WhisperEngine()
    assert e.load_model(model_path(SHAPE)) == 0 and e.is_loaded()
    return e


@pytest.mark.parametrize("vocab,ctx,lang", [
    ("DEFAULT", CTX, "en"), ("DEFAULT", None, "en"), (None, CTX, "en"), ("", CTX, "en"), ("", None, "en"),
    (None, None, "en"), ("DEFAULT", None, None)])
@pytest.mark.parametrize("clip", [0, 1])
def test_mirror_transcribe_matches_oracle(wrs, oracle, engine, vocab, ctx, lang, clip):
    vocab = wrs.DEFAULT_VOCABULARY if vocab == "DEFAULT" else vocab
    pcm = synthetic_pcm(clip, seconds=11.0)
    rc, text = engine.transcribe(pcm, lang, vocab, ctx)
    assert rc == 0
    assert text == expected_text(wrs, oracle, pcm, lang, wrs.build_initial_prompt(vocab, ctx))


def test_mirror_transcribe_chunked_matches_oracle(wrs, oracle, engine):
    """Each chunk is prompted with the vocabulary and the previous chunk's (non-empty) text."""
    chunks = [synthetic_pcm(k, seconds=11.0) for k in range(3)]
    rc, text = engine.transcribe_chunked(chunks, "en", wrs.DEFAULT_VOCABULARY)
    assert rc == 0
    results, last = [], None
    for c in chunks:
        t = expected_text(wrs, oracle, c, "en", wrs.build_initial_prompt(wrs.DEFAULT_VOCABULARY, last))
        if t:
            last = t
            results.append(t)
    assert text == " ".join(results)
    assert len(results) == 3


def test_concurrent_states_one_context(wrs):
    """Two whisper_full_with_state calls on two states of ONE context from two threads at once give
    exactly the results of the same calls made one after the other."""
    from conftest import model_path
    ctx = wrs.WhisperContext.new_with_params(model_path(SHAPE))
    clips = [synthetic_pcm(4), synthetic_pcm(5, seconds=17.0)]
    p = wrs.reference_full_params("en")

    def run(pcm, out, i):
        st = ctx.create_state()
        for _ in range(3):
            assert st.full(p, pcm) == 0
            out[i].append([([t[0] for t in s.tokens], s.t0, s.t1, s.text) for s in st.segments()])
        st.close()

    seq = [[], []]
    for i in range(2):
        run(clips[i], seq, i)
    par = [[], []]
    th = [threading.Thread(target=run, args=(clips[i], par, i)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in th)
    for i in range(2):
        assert len(par[i]) == 3
        # each call on the same state re-reads its own prompt_past: compare call by call
        assert par[i] == seq[i], i
    ctx.close()
