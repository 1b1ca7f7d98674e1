"""Generate the committed golden fixtures and pin the CPU oracle — TEST INFRASTRUCTURE ONLY.

The reference's engine (whisper.cpp via whisper-rs-sys 0.14.1) is absent offline and the
reference has no Python, so nothing from the reference itself can be run.
This script pins the oracle instead against an independent local implementation of the same
model, HF transformers' Whisper (transformers/models/whisper/modeling_whisper.py and
feature_extraction_whisper.py), on identical seeded weights:

  * mel:    oracle log-mel vs WhisperFeatureExtractor._np_extract_fbank_features (numpy STFT);
  * encoder / decoder logits: oracle mode F32 vs HF fp32 with activation gelu_pytorch_tanh.

It then records the oracle's GGML-numerics (mode 1) outputs as fixtures: mel checksum + slice,
encoder slice, prompt logits top-5, greedy token ids and segment text for the reference's
FullParams (src-tauri/src/whisper.rs:88-124). Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from make_model import SHAPES, synthetic_pcm, write_model  # noqa: E402
from oracle_py import Oracle, reference_params  # noqa: E402


def hf_model_from_ggml(path: str, shape: str):
    import torch
    from transformers import WhisperConfig, WhisperForConditionalGeneration

    n_vocab, n_mels, d, h, ne, nd = SHAPES[shape]
    cfg = WhisperConfig(vocab_size=n_vocab, num_mel_bins=n_mels, encoder_layers=ne, decoder_layers=nd,
                        encoder_attention_heads=h, decoder_attention_heads=h, d_model=d,
                        encoder_ffn_dim=4 * d, decoder_ffn_dim=4 * d, max_source_positions=1500,
                        max_target_positions=448, activation_function="gelu_pytorch_tanh",
                        dropout=0.0, attention_dropout=0.0, activation_dropout=0.0,
                        pad_token_id=50257, bos_token_id=50257, eos_token_id=50257, decoder_start_token_id=50258)
    model = WhisperForConditionalGeneration(cfg).eval()
    tensors = read_ggml_tensors(path)
    sd = {}

    def lin(dst, src, bias=True):
        sd[dst + ".weight"] = tensors[src + ".weight"]
        if bias:
            sd[dst + ".bias"] = tensors[src + ".bias"]

    sd["model.encoder.conv1.weight"] = tensors["encoder.conv1.weight"]
    sd["model.encoder.conv1.bias"] = tensors["encoder.conv1.bias"].reshape(-1)
    sd["model.encoder.conv2.weight"] = tensors["encoder.conv2.weight"]
    sd["model.encoder.conv2.bias"] = tensors["encoder.conv2.bias"].reshape(-1)
    sd["model.encoder.embed_positions.weight"] = tensors["encoder.positional_embedding"]
    for i in range(ne):
        p, q = f"encoder.blocks.{i}.", f"model.encoder.layers.{i}."
        lin(q + "self_attn.q_proj", p + "attn.query")
        lin(q + "self_attn.k_proj", p + "attn.key", bias=False)
        lin(q + "self_attn.v_proj", p + "attn.value")
        lin(q + "self_attn.out_proj", p + "attn.out")
        lin(q + "self_attn_layer_norm", p + "attn_ln")
        lin(q + "fc1", p + "mlp.0")
        lin(q + "fc2", p + "mlp.2")
        lin(q + "final_layer_norm", p + "mlp_ln")
    lin("model.encoder.layer_norm", "encoder.ln_post")
    sd["model.decoder.embed_tokens.weight"] = tensors["decoder.token_embedding.weight"]
    sd["model.decoder.embed_positions.weight"] = tensors["decoder.positional_embedding"]
    for i in range(nd):
        p, q = f"decoder.blocks.{i}.", f"model.decoder.layers.{i}."
        for a, b in (("attn", "self_attn"), ("cross_attn", "encoder_attn")):
            lin(q + b + ".q_proj", p + a + ".query")
            lin(q + b + ".k_proj", p + a + ".key", bias=False)
            lin(q + b + ".v_proj", p + a + ".value")
            lin(q + b + ".out_proj", p + a + ".out")
            lin(q + b + "_layer_norm", p + a + "_ln")
        lin(q + "fc1", p + "mlp.0")
        lin(q + "fc2", p + "mlp.2")
        lin(q + "final_layer_norm", p + "mlp_ln")
    lin("model.decoder.layer_norm", "decoder.ln")
    sd = {k: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32)) for k, v in sd.items()}
    sd["proj_out.weight"] = sd["model.decoder.embed_tokens.weight"]
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("proj_out" in k for k in missing), missing
    return model


def read_ggml_tensors(path: str) -> dict:
    import struct
    out = {}
    with open(path, "rb") as f:
        f.read(4)
        f.read(44)
        n_mel, n_fft = struct.unpack("<2i", f.read(8))
        f.read(4 * n_mel * n_fft)
        (n_tok,) = struct.unpack("<i", f.read(4))
        for _ in range(n_tok):
            (ln,) = struct.unpack("<I", f.read(4))
            f.read(ln)
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                break
            n_dims, name_len, ttype = struct.unpack("<3i", hdr)
            ne = struct.unpack(f"<{n_dims}i", f.read(4 * n_dims))
            name = f.read(name_len).decode()
            shape = tuple(reversed(ne))
            cnt = int(np.prod(shape))
            dt = np.float16 if ttype == 1 else np.float32
            out[name] = np.frombuffer(f.read(cnt * np.dtype(dt).itemsize), dtype=dt).reshape(shape).astype(np.float32)
    return out


def hf_mel(pcm: np.ndarray, n_mels: int) -> np.ndarray:
    from transformers import WhisperFeatureExtractor
    fe = WhisperFeatureExtractor(feature_size=n_mels)
    return fe._np_extract_fbank_features(pcm[None, :], "cpu")[0]


def sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def pin_against_hf(path: str, shape: str, pcm: np.ndarray) -> dict:
    """Oracle mode F32 vs HF fp32. Returns the max abs diffs (asserted by tests/test_oracle.py)."""
    import torch
    o = Oracle(path, mode=0)
    mel, _ = o.mel(pcm)
    ref = hf_mel(pcm, o.n_mels)
    d_mel = float(np.abs(mel[:, :2999] - ref[:, :2999]).max())
    hf = hf_model_from_ggml(path, shape)
    win = mel[:, :3000]
    enc = o.encode(0)
    with torch.no_grad():
        hf_enc = hf.model.encoder(torch.from_numpy(win[None])).last_hidden_state[0].numpy()
    d_enc = float(np.abs(enc - hf_enc).max())
    toks = [o.token("sot"), o.token("sot") + 1, o.token("transcribe"), o.token("beg"), 400, 1000, 77]
    o.kv_clear()
    lg = o.decode(toks, 0)
    with torch.no_grad():
        hf_lg = hf(input_features=torch.from_numpy(win[None]), decoder_input_ids=torch.tensor([toks])).logits[0].numpy()
    d_logits = float(np.abs(lg - hf_lg).max())
    o.close()
    return dict(mel_max_abs=d_mel, enc_max_abs=d_enc, logits_max_abs=d_logits,
                logits_scale=float(np.abs(hf_lg).max()))


def record_fixture(path: str, shape: str, seed: int) -> dict:
    o = Oracle(path, mode=1)
    pcm = synthetic_pcm(0)
    mel, n_len_org = o.mel(pcm)
    enc = o.encode(0)
    prompt = [o.token("sot"), o.token("sot") + 1, o.token("transcribe")] if o.n_vocab >= 51865 else [o.token("sot")]
    o.kv_clear()
    lg = o.decode(prompt, 0)[-1]
    top5 = np.argsort(-lg)[:5]
    res = o.full(pcm, reference_params("en"))
    res_prompt = o.full(pcm, reference_params("en", prompt="Claude Code, Anthropic, Supabase"))
    res_fixed = o.full(pcm, reference_params("en", fixed_tokens=32))
    tok_vocab = o.tokenize("Claude Code, Anthropic, Supabase, Vercel, shadcn, tRPC, Drizzle, Zod, pnpm, Bun")
    fx = dict(
        shape=shape, seed=seed, model_sha256=sha256(path), pcm_seed=1234,
        n_len=int(mel.shape[1]), n_len_org=int(n_len_org),
        mel_sum=float(mel.astype(np.float64).sum()), mel_slice=mel[:, :16].tolist(),
        enc_slice=enc[:8, :].tolist(),
        prompt=prompt, prompt_logits_top5=top5.tolist(), prompt_logits_top5_val=lg[top5].tolist(),
        full_en=[dict(t0=s["t0"], t1=s["t1"], text=s["text"].decode("latin-1"), tokens=s["tokens"]) for s in res["segments"]],
        full_en_no_speech=res["no_speech_prob"],
        full_prompt=[dict(t0=s["t0"], t1=s["t1"], tokens=s["tokens"]) for s in res_prompt["segments"]],
        full_fixed32=[dict(t0=s["t0"], t1=s["t1"], tokens=s["tokens"]) for s in res_fixed["segments"]],
        tokenize_vocab=tok_vocab,
    )
    o.close()
    return fx


def main():
    out = {}
    os.makedirs("/tmp/nw_golden", exist_ok=True)
    for shape, seed in (("micro", 0), ("tiny", 0)):
        path = f"/tmp/nw_golden/{shape}_s{seed}.bin"
        write_model(path, shape, seed)
        pin = pin_against_hf(path, shape, synthetic_pcm(0))
        print(shape, "HF pin:", pin)
        fx = record_fixture(path, shape, seed)
        fx["hf_pin"] = pin
        out[f"{shape}_s{seed}"] = fx
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
