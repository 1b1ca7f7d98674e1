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
