"""The C++ mirror of the reference's boundary caller (src-tauri/src/whisper.rs) — CPU only."""
import pytest


def test_filter_hallucinations_known_answers(wrs):
    # src-tauri/src/whisper.rs:285-305 (test_filter_hallucinations), verbatim cases
    f = wrs.filter_hallucinations
    assert f("Thank you for watching!") == ""
    assert f("thanks for watching.") == ""
    assert f("Thank you for watching") == ""
    assert f("Subscribe to my channel") == ""
    assert f("you") == ""
    assert f("...") == ""
    assert f("시청해 주셔서 감사합니다") == ""
    assert f("Hello, this is a real sentence.") == "Hello, this is a real sentence."
    assert f("Thank you for watching the demo, now let me explain") == \
        "Thank you for watching the demo, now let me explain"


def test_filter_hallucinations_edges(wrs):
    f = wrs.filter_hallucinations
    assert f("   ") == ""
    assert f("  hello  ") == "hello"
    assert f("♪ ♪") == "♪ ♪"          # space is not punctuation: passes (as in Rust)
    assert f("♪♪…") == ""
    assert f("MBC 뉴스 이덕영입니다") == ""
    assert f("mbc 뉴스 이덕영입니다!!") == ""
    assert f("YOU...") == ""
    assert f("you know") == "you know"


def test_engine_new_not_loaded(wrs):
    # whisper.rs:272-276 test_whisper_engine_new
    e = wrs.WhisperEngine()
    assert not e.is_loaded()


def test_transcribe_without_model(wrs):
    # whisper.rs:278-283 test_transcribe_without_model: 1 s of zeros -> NoModel
    import numpy as np
    e = wrs.WhisperEngine()
    rc, text = e.transcribe(np.zeros(16000, np.float32))
    assert rc == wrs.WhisperEngine.NO_MODEL and text is None


@pytest.mark.parametrize("vocab,ctx,expected", [
    ("Claude Code, Anthropic", "previous text", "Claude Code, Anthropic previous text"),  # (Some(v), Some(c)) if !v.is_empty()
    ("Claude Code, Anthropic", None, "Claude Code, Anthropic"),                           # (Some(v), None) if !v.is_empty()
    (None, "previous text", "previous text"),                                             # (_, Some(c))
    ("", "previous text", "previous text"),                                               # empty vocab falls to (_, Some(c))
    ("", None, None),                                                                     # _ => None
    (None, None, None),
    ("vocab", "", "vocab "),                                                              # Some("") context is still Some
])
def test_initial_prompt_branches(wrs, vocab, ctx, expected):
    """whisper.rs:98-105: the four match arms of the initial-prompt assembly."""
    assert wrs.build_initial_prompt(vocab, ctx) == expected


def test_utf8_lossy_matches_rust_semantics(wrs):
    """segment.to_str_lossy() (whisper.rs:137) is String::from_utf8_lossy: each maximal ill-formed
    subsequence becomes one U+FFFD. Python's 'replace' handler implements the same Unicode
    practice, so it is the reference here (fuzzed over segment-edge splits of multi-byte chars)."""
    import random
    rng = random.Random(0)
    pieces = [b"\xe2\x82", b"\xf0\x9f\x98\x80", b"\xed\xa0\x80", b"\xc0\xaf", b"\xf4\x90\x80\x80", b"a", b" ",
              b"\xe6\x84\x9f", b"\x80", b"\xff", b"\xf0\x80\x80", b"\xe0\x80\xaf", b"\xc2", b"\xec\x8b\x9c"]
    for _ in range(5000):
        s = b"".join(rng.choice(pieces) for _ in range(rng.randint(0, 10)))
        assert wrs.utf8_lossy(s) == s.decode("utf-8", "replace").encode(), s
    # a character split across two segments: each half is replaced separately (not re-joined)
    full = "감사".encode()
    assert wrs.utf8_lossy(full[:2]) + wrs.utf8_lossy(full[2:]) == "\ufffd\ufffd사".encode()
