"""Seeded synthetic Whisper models in the GGML `.bin` layout that whisper.cpp reads.

No real weights exist offline, so every parity test, golden fixture and
bench run uses a file written by this tool. The byte layout is the one the reference app
stores as `ggml-<id>.bin` (src-tauri/src/model.rs:190-198, lib.rs:29) and that whisper.cpp's
loader parses [ext, whisper.cpp ≈v1.7.x `whisper_model_load`, written by its
`models/convert-pt-to-ggml.py`]:

  u32  magic 0x67676d6c
  i32  n_vocab n_audio_ctx n_audio_state n_audio_head n_audio_layer
       n_text_ctx n_text_state n_text_head n_text_layer n_mels ftype
  i32  n_mel, n_fft(=201); f32 filters[n_mel][n_fft]
  i32  n_tokens; per token: u32 len, bytes
  tensors: i32 n_dims, i32 name_len, i32 ttype, i32 ne[n_dims] (innermost first), name, data

Tensor names are OpenAI-Whisper names; 1-D tensors, conv biases and positional embeddings
are f32, every other tensor is f16 (ftype 1), exactly as convert-pt-to-ggml.py writes them.
"""
from __future__ import annotations

import argparse
import os
import struct

import numpy as np

GGML_MAGIC = 0x67676D6C

# Standard Whisper shapes plus a "micro" shape that keeps the CPU oracle
# fast enough to run the whole whisper_full control loop inside unit tests.
SHAPES = {
    #            n_vocab n_mels  d    h  Le  Ld
    "micro":    (51865, 80,   64,  1, 1, 1),
    "tiny.en":  (51864, 80,  384,  6, 4, 4),
    "tiny":     (51865, 80,  384,  6, 4, 4),
    "base":     (51865, 80,  512,  8, 6, 6),
    "small":    (51865, 80,  768, 12, 12, 12),
    "medium":   (51865, 80, 1024, 16, 24, 24),
    "large-v3": (51866, 128, 1280, 20, 32, 32),
    "large-v3-turbo": (51866, 128, 1280, 20, 32, 4),
    # BASELINE config shapes at reduced depth (real d / heads / n_mels / n_vocab), so that the CPU
    # oracle runs a whole whisper_full in seconds inside the parity tests
    "small-4L": (51865, 80, 768, 12, 4, 4),
    "large-v3-2L": (51866, 128, 1280, 20, 2, 2),
    "large-v3-turbo-2L": (51866, 128, 1280, 20, 2, 4),
    # one encoder and one decoder layer at small's width (kernel debugging: every buffer of a decode step is
    # the one layer's)
    "small-1L": (51865, 80, 768, 12, 1, 1),
}

# "+conf" variant: a decoder whose output distribution is as peaked as a trained model's (random
# weights give near-flat logits, avg logprob ~ -6, so every window falls back to sampled t > 0
# attempts). decoder.ln is scaled (logit std ~ CONF_SCALE), column 0 of the final LN output is a
# constant 1 and the timestamp rows of the token embedding carry CONF_TS_BOOST there (timestamps
# compete with text, so windows end on timestamp pairs), and the decoder positional embedding is
# CONF_POS_SCALE x larger (the greedy sequence does not cycle, entropy stays above 2.4). With the
# reference's FullParams the greedy t = 0 attempt then passes the fallback thresholds.
CONF_SCALE, CONF_TS_BOOST, CONF_POS_SCALE = 6.0, 14.0, 10.0
# "+conf+eot": the same, and the EOT row carries CONF_EOT_BOOST in column 0, so EOT competes with the top text
# tokens and windows decoded with no_timestamps end at steps that differ from clip to clip (tests of the
# pipelined decoding with rows at different steps, tests/test_gpu_pipe.py)
CONF_EOT_BOOST = 18.0


def token_beg(n_vocab: int) -> int:
    """whisper.cpp's token_beg for a vocabulary size (special ids shift in multilingual files)."""
    if n_vocab < 51865:
        return 50363
    return 50363 + (n_vocab - 51765 - 1) - 98

N_AUDIO_CTX = 1500
N_TEXT_CTX = 448
N_FFT_BINS = 201
N_BASE_TOKENS = 50257  # GPT-2 byte-level tokens incl. <|endoftext|>; specials are added by the loader


def mel_filters_slaney(n_mels: int, sr: int = 16000, n_fft: int = 400) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, htk=False, norm='slaney') — the filterbank that
    OpenAI Whisper's mel_filters.npz holds and convert-pt-to-ggml.py copies into the file."""
    def hz_to_mel(f):
        f = np.asanyarray(f, dtype=np.float64)
        f_sp = 200.0 / 3
        mels = f / f_sp
        min_log_hz = 1000.0
        min_log_mel = min_log_hz / f_sp
        logstep = np.log(6.4) / 27.0
        return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)

    def mel_to_hz(m):
        m = np.asanyarray(m, dtype=np.float64)
        f_sp = 200.0 / 3
        freqs = f_sp * m
        min_log_hz = 1000.0
        min_log_mel = min_log_hz / f_sp
        logstep = np.log(6.4) / 27.0
        return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)

    fftfreqs = np.linspace(0, sr / 2, 1 + n_fft // 2)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(sr / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    weights = np.zeros((n_mels, len(fftfreqs)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, None]
    return weights.astype(np.float32)


def synthetic_vocab(seed: int = 7) -> list[bytes]:
    """50257 unique byte strings standing in for the GPT-2 vocabulary (not shipped offline).

    Ids 0..255 are single bytes (so greedy longest-prefix tokenisation always succeeds),
    then English-like sub-words with and without a leading space, then seeded random
    letter strings. Id 50256 is <|endoftext|> as in the real file."""
    rng = np.random.default_rng(seed)
    toks: list[bytes] = [bytes([b]) for b in range(256)]
    seen = set(toks)

    def add(t: bytes):
        if t not in seen and len(toks) < N_BASE_TOKENS - 1:
            seen.add(t)
            toks.append(t)

    words = (
        "the of and to in is you that it he was for on are as with his they at be this have from "
        "or one had by word but not what all were we when your can said there use an each which she "
        "do how their if will up other about out many then them these so some her would make like him "
        "into time has look two more write go see number no way could people my than first water been "
        "call who oil its now find long down day did get come made may part code claude anthropic "
        "supabase vercel shadcn trpc drizzle zod pnpm bun deno turso neon planetscale turborepo tauri "
        "sveltekit nuxt astro vite zustand tanstack langchain llamaindex ollama cursor neovim vitest "
        "playwright prisma radix fly io railway cloudflare workers hono htmx biome oxlint rspack "
        "turbopack qwik solidjs convex upstash resend inngest replit v0 lovable bolt windsurf codeium "
        "supermaven aider openrouter perplexity groq mistral cohere replicate hello world thank watching"
    ).split()
    for w in words:
        for v in (w, w.capitalize(), w.upper()):
            add(v.encode())
            add(b" " + v.encode())
    for p in [",", ".", "!", "?", "'s", "'t", "'re", "'ve", "'m", "'ll", "'d", " -", "...", " ...", "\n"]:
        add(p.encode())
    letters = "abcdefghijklmnopqrstuvwxyz"
    for a in letters:
        for b in letters:
            add((a + b).encode())
            add((" " + a + b).encode())
    while len(toks) < N_BASE_TOKENS - 1:
        n = int(rng.integers(3, 9))
        s = "".join(letters[i] for i in rng.integers(0, 26, n))
        if rng.random() < 0.5:
            s = " " + s
        add(s.encode())
    toks.append(b"<|endoftext|>")
    assert len(toks) == N_BASE_TOKENS and len(set(toks)) == N_BASE_TOKENS
    return toks


def sinusoids(length: int, channels: int, max_timescale: float = 10000) -> np.ndarray:
    """Whisper's encoder positional embedding (openai/whisper model.py `sinusoids`)."""
    log_timescale_increment = np.log(max_timescale) / (channels // 2 - 1)
    inv_timescales = np.exp(-log_timescale_increment * np.arange(channels // 2))
    scaled_time = np.arange(length)[:, None] * inv_timescales[None, :]
    return np.concatenate([np.sin(scaled_time), np.cos(scaled_time)], axis=1).astype(np.float32)


def tensor_specs(n_vocab, n_mels, d, n_enc, n_dec):
    """(name, pytorch-shape, f32?) in the order convert-pt-to-ggml.py emits them."""
    specs = [
        ("encoder.positional_embedding", (N_AUDIO_CTX, d), True),
        ("encoder.conv1.weight", (d, n_mels, 3), False),
        ("encoder.conv1.bias", (d, 1), True),
        ("encoder.conv2.weight", (d, d, 3), False),
        ("encoder.conv2.bias", (d, 1), True),
    ]
    for i in range(n_enc):
        p = f"encoder.blocks.{i}."
        specs += [
            (p + "attn.query.weight", (d, d), False), (p + "attn.query.bias", (d,), True),
            (p + "attn.key.weight", (d, d), False),
            (p + "attn.value.weight", (d, d), False), (p + "attn.value.bias", (d,), True),
            (p + "attn.out.weight", (d, d), False), (p + "attn.out.bias", (d,), True),
            (p + "attn_ln.weight", (d,), True), (p + "attn_ln.bias", (d,), True),
            (p + "mlp.0.weight", (4 * d, d), False), (p + "mlp.0.bias", (4 * d,), True),
            (p + "mlp.2.weight", (d, 4 * d), False), (p + "mlp.2.bias", (d,), True),
            (p + "mlp_ln.weight", (d,), True), (p + "mlp_ln.bias", (d,), True),
        ]
    specs += [("encoder.ln_post.weight", (d,), True), ("encoder.ln_post.bias", (d,), True)]
    specs += [
        ("decoder.positional_embedding", (N_TEXT_CTX, d), True),
        ("decoder.token_embedding.weight", (n_vocab, d), False),
    ]
    for i in range(n_dec):
        p = f"decoder.blocks.{i}."
        for a in ("attn", "cross_attn"):
            specs += [
                (p + a + ".query.weight", (d, d), False), (p + a + ".query.bias", (d,), True),
                (p + a + ".key.weight", (d, d), False),
                (p + a + ".value.weight", (d, d), False), (p + a + ".value.bias", (d,), True),
                (p + a + ".out.weight", (d, d), False), (p + a + ".out.bias", (d,), True),
                (p + a + "_ln.weight", (d,), True), (p + a + "_ln.bias", (d,), True),
            ]
        specs += [
            (p + "mlp.0.weight", (4 * d, d), False), (p + "mlp.0.bias", (4 * d,), True),
            (p + "mlp.2.weight", (d, 4 * d), False), (p + "mlp.2.bias", (d,), True),
            (p + "mlp_ln.weight", (d,), True), (p + "mlp_ln.bias", (d,), True),
        ]
    specs += [("decoder.ln.weight", (d,), True), ("decoder.ln.bias", (d,), True)]
    return specs


def init_tensor(rng, name, shape, d, n_mels):
    if name == "encoder.positional_embedding":
        return sinusoids(N_AUDIO_CTX, d)
    if name.endswith("_ln.weight") or name.endswith("ln_post.weight") or name == "decoder.ln.weight":
        return (1.0 + 0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name.endswith(".bias"):
        return (0.05 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name == "decoder.positional_embedding":
        return (0.1 * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)
    if name == "decoder.token_embedding.weight":
        std = 1.0 / np.sqrt(d)
    elif name.startswith("encoder.conv1"):
        std = 1.0 / np.sqrt(n_mels * 3)
    elif name.startswith("encoder.conv2"):
        std = 1.0 / np.sqrt(d * 3)
    else:
        std = 1.0 / np.sqrt(shape[1])  # linear [out, in]: fan-in
    return (std * rng.standard_normal(shape, dtype=np.float32)).astype(np.float32)


def conf_adjust(name: str, t: np.ndarray, n_vocab: int, eot_boost: float = 0.0) -> np.ndarray:
    if name in ("decoder.ln.weight", "decoder.ln.bias"):
        t = t * CONF_SCALE
        t[0] = 0.0 if name.endswith("weight") else 1.0
    elif name == "decoder.token_embedding.weight":
        t[:, 0] = 0.0
        t[token_beg(n_vocab):, 0] = CONF_TS_BOOST
        if eot_boost:
            t[50256 + (n_vocab >= 51865), 0] = eot_boost  # token_eot (multilingual vocabularies shift it by one)
    elif name == "decoder.positional_embedding":
        t = t * CONF_POS_SCALE
    return t


# ---- GGML block quantization (the app's catalog ships small-q5_1, medium-q5_0 and large-v3-q5_0:
# src-tauri/src/model.rs:153-186). Tensor type ids and block layouts of ggml [ext, ggml-common.h]:
#   Q4_0 = 2: {f16 d; u8 qs[16]}            18 B / 32      Q4_1 = 3: {f16 d, m; u8 qs[16]}        20 B / 32
#   Q5_0 = 6: {f16 d; u8 qh[4]; u8 qs[16]}   22 B / 32      Q5_1 = 7: {f16 d, m; u8 qh[4]; qs[16]} 24 B / 32
#   Q8_0 = 8: {f16 d; i8 qs[32]}             34 B / 32
# The file's ftype is GGML_FTYPE_MOSTLY_* + 1000 * GGML_QNT_VERSION (2). whisper.cpp's quantize tool
# quantizes every 2-D tensor except the positional embeddings (3-D conv weights and 1-D tensors stay).
GGML_TYPES = {"q4_0": 2, "q4_1": 3, "q5_0": 6, "q5_1": 7, "q8_0": 8}
GGML_FTYPES = {"q4_0": 2, "q4_1": 3, "q5_0": 8, "q5_1": 9, "q8_0": 7}
GGML_QNT_VERSION = 2
# whisper.cpp's quantize tool: 2-D tensors only, minus these (examples/quantize, to_skip) [ext]
QUANT_SKIP = ("encoder.conv1.bias", "encoder.conv2.bias", "encoder.positional_embedding",
              "decoder.positional_embedding")
BLOCK_BYTES = {2: 18, 3: 20, 6: 22, 7: 24, 8: 34}


def read_tensors(path: str) -> dict:
    """Parse a GGML whisper file: {name: (ggml type, ne (innermost first), raw bytes)}."""
    with open(path, "rb") as f:
        buf = f.read()
    o = 4 + 11 * 4
    n_mel, n_fft = struct.unpack_from("<2i", buf, o)
    o += 8 + 4 * n_mel * n_fft
    (n_tok,) = struct.unpack_from("<i", buf, o)
    o += 4
    for _ in range(n_tok):
        (ln,) = struct.unpack_from("<I", buf, o)
        o += 4 + ln
    out = {}
    while o < len(buf):
        nd, nl, tt = struct.unpack_from("<3i", buf, o)
        o += 12
        ne = struct.unpack_from(f"<{nd}i", buf, o)
        o += 4 * nd
        name = buf[o:o + nl].decode()
        o += nl
        nel = int(np.prod(ne))
        nbytes = nel * 4 if tt == 0 else nel * 2 if tt == 1 else nel // 32 * BLOCK_BYTES[tt]
        out[name] = (tt, ne, buf[o:o + nbytes])
        o += nbytes
    return out


def quantize_rows(x: np.ndarray, qtype: str) -> bytes:
    """ggml's quantize_row_*_reference over the rows of x (row length % 32 == 0), vectorised."""
    b = x.astype(np.float32).reshape(-1, 32)
    nb = b.shape[0]
    if qtype in ("q5_0", "q4_0"):
        nmax = 16 if qtype == "q5_0" else 8
        am = np.abs(b).argmax(1)
        mx = b[np.arange(nb), am]
        d = mx / -nmax
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        q = np.minimum(2 * nmax - 1, (b * idd[:, None] + np.float32(nmax + 0.5)).astype(np.int8)).astype(np.int32)
        dh = d.astype(np.float16).view(np.uint16)
    elif qtype in ("q5_1", "q4_1"):
        lo, hi = b.min(1), b.max(1)
        d = (hi - lo) / (31 if qtype == "q5_1" else 15)
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        q = ((b - lo[:, None]) * idd[:, None] + np.float32(0.5)).astype(np.uint8).astype(np.int32)
        q = np.minimum(q, 31 if qtype == "q5_1" else 15)
        dh = d.astype(np.float16).view(np.uint16)
        mh = lo.astype(np.float16).view(np.uint16)
    else:  # q8_0
        amax = np.abs(b).max(1)
        d = amax / 127
        idd = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0).astype(np.float32)
        q = np.round(b * idd[:, None]).astype(np.int8)
        dh = d.astype(np.float16).view(np.uint16)
        return b"".join(dh[i].tobytes() + q[i].tobytes() for i in range(nb))
    qs = ((q[:, :16] & 0x0F) | ((q[:, 16:] & 0x0F) << 4)).astype(np.uint8)
    out = []
    if qtype in ("q5_0", "q5_1"):
        hb = ((q >> 4) & 1).astype(np.uint64)
        qh = (hb << np.arange(32, dtype=np.uint64)).sum(1).astype(np.uint32)
    for i in range(nb):
        rec = dh[i].tobytes()
        if qtype in ("q5_1", "q4_1"):
            rec += mh[i].tobytes()
        if qtype in ("q5_0", "q5_1"):
            rec += qh[i].tobytes()
        out.append(rec + qs[i].tobytes())
    return b"".join(out)


def dequantize_rows(raw: bytes, qtype: str, n: int) -> np.ndarray:
    """ggml's dequantize_row_* (f32 results: q*d (+ m), the product exact in f32)."""
    bs = {"q4_0": 18, "q4_1": 20, "q5_0": 22, "q5_1": 24, "q8_0": 34}[qtype]
    a = np.frombuffer(raw, np.uint8).reshape(-1, bs)
    d = a[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
    if qtype == "q8_0":
        return (a[:, 2:].view(np.int8).astype(np.float32) * d[:, None]).reshape(-1)[:n]
    off = 2
    m = None
    if qtype in ("q5_1", "q4_1"):
        m = a[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
        off = 4
    qh = None
    if qtype in ("q5_0", "q5_1"):
        qh = a[:, off:off + 4].copy().view(np.uint32)[:, 0].astype(np.uint64)
        off += 4
    qs = a[:, off:off + 16].astype(np.int32)
    q = np.concatenate([qs & 0x0F, qs >> 4], 1)
    if qh is not None:
        q = q | ((((qh[:, None] >> np.arange(32, dtype=np.uint64)) & 1).astype(np.int32)) << 4)
    if m is None:
        q = q - (16 if qtype == "q5_0" else 8)
        y = q.astype(np.float32) * d[:, None]
    else:
        y = q.astype(np.float32) * d[:, None] + m[:, None]
    return y.reshape(-1)[:n]


def write_model(path: str, shape: str = "tiny", seed: int = 0, ftype: int = 1, qtype: str | None = None,
                progress=None) -> dict:
    """Write a seeded synthetic model. Returns the hparams dict. ftype 1 = f16 matrices, 0 = all f32.
    shape may carry the "+conf" suffix (see CONF_SCALE) and a "+q5_0" / "+q5_1" / "+q8_0" / "+q4_0" /
    "+q4_1" suffix: every 2-D tensor but QUANT_SKIP quantized as whisper.cpp's quantize tool does.
    progress(name), if given, is called before every tensor (long writes can report that they move)."""
    for q in GGML_TYPES:
        if shape.endswith("+" + q):
            shape, qtype = shape[:-len(q) - 1], q
    eot = shape.endswith("+eot")
    if eot:
        shape = shape[:-4]
    conf = shape.endswith("+conf")
    n_vocab, n_mels, d, h, n_enc, n_dec = SHAPES[shape[:-5] if conf else shape]
    rng = np.random.default_rng(seed)
    hp = dict(n_vocab=n_vocab, n_audio_ctx=N_AUDIO_CTX, n_audio_state=d, n_audio_head=h,
              n_audio_layer=n_enc, n_text_ctx=N_TEXT_CTX, n_text_state=d, n_text_head=h,
              n_text_layer=n_dec, n_mels=n_mels,
              ftype=ftype if qtype is None else GGML_FTYPES[qtype] + 1000 * GGML_QNT_VERSION)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<I", GGML_MAGIC))
        f.write(struct.pack("<11i", *hp.values()))
        filt = mel_filters_slaney(n_mels)
        f.write(struct.pack("<2i", n_mels, N_FFT_BINS))
        f.write(filt.astype("<f4").tobytes())
        toks = synthetic_vocab()
        f.write(struct.pack("<i", len(toks)))
        for t in toks:
            f.write(struct.pack("<I", len(t)))
            f.write(t)
        for name, shp, is_f32 in tensor_specs(n_vocab, n_mels, d, n_enc, n_dec):
            if progress is not None:
                progress(name)
            data = init_tensor(rng, name, shp, d, n_mels)
            if conf:
                data = conf_adjust(name, data, n_vocab, CONF_EOT_BOOST if eot else 0.0)
            use_f16 = (ftype == 1) and not is_f32
            quant = qtype is not None and len(shp) == 2 and name not in QUANT_SKIP
            nb = name.encode()
            ttype = GGML_TYPES[qtype] if quant else (1 if use_f16 else 0)
            f.write(struct.pack("<3i", len(shp), len(nb), ttype))
            f.write(struct.pack(f"<{len(shp)}i", *reversed(shp)))
            f.write(nb)
            if quant:
                f.write(quantize_rows(data, qtype))
            else:
                f.write(data.astype("<f2" if use_f16 else "<f4").tobytes())
    os.replace(tmp, path)
    return hp


def synthetic_pcm(k: int, seconds: float = 30.0, sr: int = 16000) -> np.ndarray:
    """SURVEY.md §8d synthetic chunk k (seed 1234+k): 3-5 amplitude-modulated harmonic stacks
    (100-3000 Hz) separated by 0.7-1.0 s silences, plus Gaussian noise at RMS 0.005, peak ~0.3."""
    rng = np.random.default_rng(1234 + k)
    n = int(seconds * sr)
    t = np.arange(n, dtype=np.float64) / sr
    x = np.zeros(n, dtype=np.float64)
    nseg = int(rng.integers(3, 6))
    pos = 0.0
    seg_len = seconds / nseg
    for _ in range(nseg):
        sil = float(rng.uniform(0.7, 1.0))
        start, end = pos + sil, min(pos + seg_len, seconds)
        if end > start:
            f0 = float(rng.uniform(100, 300))
            m = (t >= start) & (t < end)
            tone = np.zeros(m.sum())
            for hmul in range(1, int(rng.integers(3, 8))):
                f = f0 * hmul
                if f > 3000:
                    break
                tone += np.sin(2 * np.pi * f * t[m] + rng.uniform(0, 2 * np.pi)) / hmul
            am = 0.5 * (1 + np.sin(2 * np.pi * rng.uniform(2, 6) * t[m]))
            x[m] += tone * am
        pos += seg_len
    if np.abs(x).max() > 0:
        x *= 0.3 / np.abs(x).max()
    x += 0.005 * rng.standard_normal(n)
    return x.astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--shape", default="tiny", help="a SHAPES key, optionally +conf and/or +q5_0 / +q5_1 / +q8_0 / +q4_0 / +q4_1")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--ftype", type=int, default=1)
    a = ap.parse_args()
    print(write_model(a.out, a.shape, a.seed, a.ftype))


if __name__ == "__main__":
    main()
