"""CPU oracle checks (no GPU): the restated whisper.cpp algorithm against the committed golden
fixtures and the HF-transformers pin recorded by tests/golden/make_golden.py."""
import numpy as np
import pytest

from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params


@pytest.fixture(scope="module")
def tiny_oracle(tiny_model):
    o = Oracle(tiny_model, mode=1)
    yield o
    o.close()


def test_model_file_is_deterministic(tiny_model, golden):
    import hashlib
    with open(tiny_model, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    assert digest == golden["tiny_s0"]["model_sha256"]


def test_hf_pin_recorded(golden):
    # oracle (F32 mode) vs HF transformers Whisper fp32 on identical weights
    for key in ("micro_s0", "tiny_s0"):
        pin = golden[key]["hf_pin"]
        assert pin["mel_max_abs"] < 1e-4
        assert pin["enc_max_abs"] < 2e-3
        assert pin["logits_max_abs"] < 2e-3 * max(1.0, pin["logits_scale"])


def test_mel_matches_golden(tiny_oracle, golden):
    g = golden["tiny_s0"]
    mel, n_len_org = tiny_oracle.mel(synthetic_pcm(0))
    assert mel.shape[1] == g["n_len"] and n_len_org == g["n_len_org"]
    np.testing.assert_array_equal(mel[:, :16], np.array(g["mel_slice"], np.float32))
    assert abs(float(mel.astype(np.float64).sum()) - g["mel_sum"]) < 1e-6


def test_encoder_matches_golden(tiny_oracle, golden):
    tiny_oracle.mel(synthetic_pcm(0))
    enc = tiny_oracle.encode(0)
    np.testing.assert_allclose(enc[:8], np.array(golden["tiny_s0"]["enc_slice"], np.float32), rtol=0, atol=2e-5)


def test_prompt_logits_top5(tiny_oracle, golden):
    g = golden["tiny_s0"]
    tiny_oracle.mel(synthetic_pcm(0))
    tiny_oracle.encode(0)
    tiny_oracle.kv_clear()
    lg = tiny_oracle.decode(g["prompt"], 0)[-1]
    assert np.argsort(-lg)[:5].tolist() == g["prompt_logits_top5"]


def test_full_matches_golden_micro(micro_model, golden):
    o = Oracle(micro_model, mode=1)
    r = o.full(synthetic_pcm(0), reference_params("en"))
    got = [s["tokens"] for s in r["segments"]]
    assert got == [s["tokens"] for s in golden["micro_s0"]["full_en"]]
    o.close()


def test_tokenizer_golden(tiny_oracle, golden):
    t = tiny_oracle.tokenize("Claude Code, Anthropic, Supabase, Vercel, shadcn, tRPC, Drizzle, Zod, pnpm, Bun")
    assert t == golden["tiny_s0"]["tokenize_vocab"]
    # greedy longest match: every token re-joins to the input
    assert b"".join(tiny_oracle.token_str(i) for i in t) == b"Claude Code, Anthropic, Supabase, Vercel, shadcn, tRPC, Drizzle, Zod, pnpm, Bun"


def test_mel_short_and_empty_inputs(tiny_oracle):
    # 0.5 s, odd length, and a >30 s clip: n_len / n_len_org follow whisper.cpp's formulas
    for n in (8000, 16001, 16000 * 45 + 7):
        mel, org = tiny_oracle.mel(np.random.default_rng(n).standard_normal(n).astype(np.float32) * 0.1)
        assert mel.shape[1] == (n + 480000) // 160
        assert org == 1 + (n + 200 - 400) // 160
        assert np.isfinite(mel).all()
        assert mel.max() <= (mel.max() + 4) and mel.min() >= mel.max() - 2.0 - 1e-6
