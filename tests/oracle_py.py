"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the
product path (nobs-whisper_amd/) never imports or links it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")


class Decision(C.Structure):
    """State::Decision == struct whisper_mi355x_window_decision (include/whisper_mi355x.h)."""
    _fields_ = [("seek", C.c_int32), ("temp_idx", C.c_int32), ("failed0", C.c_int32), ("logprob_fail0", C.c_int32),
                ("result_len0", C.c_int32), ("no_speech", C.c_int32), ("avg_logprob0", C.c_float),
                ("entropy0", C.c_float), ("no_speech_prob", C.c_float), ("pad", C.c_float)]


def decisions_to_dicts(arr) -> list:
    return [{f: getattr(d, f) for f, _ in Decision._fields_ if f != "pad"} for d in arr]


class OracleParams(C.Structure):
    _fields_ = [
        ("language", C.c_char_p), ("initial_prompt", C.c_char_p),
        ("n_max_text_ctx", C.c_int), ("offset_ms", C.c_int), ("duration_ms", C.c_int),
        ("translate", C.c_int), ("no_context", C.c_int), ("no_timestamps", C.c_int),
        ("single_segment", C.c_int), ("print_special", C.c_int), ("suppress_blank", C.c_int),
        ("max_tokens", C.c_int),
        ("temperature", C.c_float), ("temperature_inc", C.c_float), ("max_initial_ts", C.c_float),
        ("length_penalty", C.c_float), ("entropy_thold", C.c_float), ("logprob_thold", C.c_float),
        ("no_speech_thold", C.c_float),
        ("best_of", C.c_int), ("fixed_tokens", C.c_int),
    ]


def reference_params(language: str | None = "en", prompt: str | None = None, fixed_tokens: int = 0) -> OracleParams:
    """whisper_full_default_params(GREEDY) + the setters of src-tauri/src/whisper.rs:88-124."""
    p = OracleParams()
    p.language = language.encode() if language else None
    p.initial_prompt = prompt.encode() if prompt else None
    p.n_max_text_ctx = 16384
    p.offset_ms = p.duration_ms = 0
    p.translate = 0; p.no_context = 0; p.no_timestamps = 0; p.single_segment = 0
    p.print_special = 0; p.suppress_blank = 1; p.max_tokens = 0
    p.temperature = 0.0; p.temperature_inc = 0.2; p.max_initial_ts = 1.0; p.length_penalty = -1.0
    p.entropy_thold = 2.4; p.logprob_thold = -1.0; p.no_speech_thold = 0.6
    p.best_of = 1
    p.fixed_tokens = fixed_tokens
    return p


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, ip, fp = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_float)
        sig = {
            "oracle_load": (vp, [C.c_char_p, C.c_int, C.c_int]),
            "oracle_free": (None, [vp]),
            "oracle_set_threads": (None, [vp, C.c_int]),
            "oracle_state_new": (vp, [vp]),
            "oracle_state_free": (None, [vp]),
            "oracle_token": (C.c_int, [vp, C.c_char_p]),
            "oracle_mel": (C.c_int, [vp, vp, fp, C.c_int, ip]),
            "oracle_state_mel": (None, [vp, fp]),
            "oracle_set_mel": (None, [vp, vp, fp, C.c_int]),
            "oracle_encode": (None, [vp, vp, C.c_int, fp]),
            "oracle_cross_kv": (None, [vp, vp, C.c_int, fp, fp]),
            "oracle_kv_clear": (None, [vp]),
            "oracle_decode": (None, [vp, vp, ip, C.c_int, C.c_int, fp]),
            "oracle_tokenize": (C.c_int, [vp, C.c_char_p, ip, C.c_int]),
            "oracle_token_str": (C.c_char_p, [vp, C.c_int]),
            "oracle_lang_detect": (C.c_int, [vp, vp]),
            "oracle_full": (C.c_int, [vp, vp, C.POINTER(OracleParams), fp, C.c_int]),
            "oracle_n_segments": (C.c_int, [vp]),
            "oracle_segment_text": (C.c_char_p, [vp, C.c_int]),
            "oracle_segment_t": (None, [vp, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
            "oracle_segment_n_tokens": (C.c_int, [vp, C.c_int]),
            "oracle_segment_token": (C.c_int, [vp, C.c_int, C.c_int]),
            "oracle_lang": (C.c_int, [vp]),
            "oracle_no_speech": (C.c_float, [vp]),
            "oracle_n_steps": (C.c_int, [vp]),
            "oracle_n_decisions": (C.c_int, [vp]),
            "oracle_decisions": (None, [vp, vp]),
            "oracle_step_margins": (None, [vp, fp]),
            "oracle_step_tokens": (None, [vp, ip, ip]),
            "oracle_segment_seek": (C.c_int, [vp, C.c_int]),
            "oracle_step_logits": (C.c_long, [vp, vp, fp, C.c_long]),
            "oracle_decoder_tokens": (C.c_int, [vp, ip, C.c_int]),
            "oracle_mel_tables": (None, [fp, fp, fp]),
            "oracle_tensor": (C.c_long, [vp, C.c_char_p, C.c_int, fp, C.c_long]),
            "oracle_calculate_rms": (C.c_float, [fp, C.c_int]),
            "oracle_estimate_noise_floor": (C.c_float, [fp, C.c_int, C.c_int]),
            "oracle_find_silence_boundaries": (C.c_int, [fp, C.c_int, C.c_int, ip, C.c_int]),
            "oracle_split_at_silences": (C.c_int, [C.c_int, ip, C.c_int, C.c_int, ip, ip, C.c_int]),
            "oracle_resample": (C.c_int, [fp, C.c_int, C.c_int, fp, C.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Oracle:
    """One loaded model + one state (mirrors whisper_context + whisper_state)."""

    def __init__(self, path: str, mode: int = 1, n_threads: int = 8):
        self.L = lib()
        self.m = self.L.oracle_load(path.encode(), mode, n_threads)
        if not self.m:
            raise RuntimeError(f"oracle failed to load {path}")
        self.s = self.L.oracle_state_new(self.m)
        import struct
        with open(path, "rb") as f:
            f.read(4)
            hp = struct.unpack("<11i", f.read(44))
        (self.n_vocab, self.n_audio_ctx, self.d, self.n_head, self.n_enc, self.n_text_ctx, _, _,
         self.n_dec, self.n_mels, _) = hp

    def new_state(self):
        """A fresh whisper_state (whisper.rs:83-85 creates one per transcribe call): empty
        prompt_past, rng re-seeded."""
        self.L.oracle_state_free(self.s)
        self.s = self.L.oracle_state_new(self.m)

    def close(self):
        if self.m:
            self.L.oracle_state_free(self.s)
            self.L.oracle_free(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tensor(self, name: str, lookup: bool = False) -> np.ndarray:
        """A loaded tensor as the oracle computes with it (flat, ggml element order)."""
        n = self.L.oracle_tensor(self.m, name.encode(), int(lookup), None, 0)
        if n < 0:
            raise KeyError(name)
        out = np.empty(n, np.float32)
        self.L.oracle_tensor(self.m, name.encode(), int(lookup), _fp(out), n)
        return out

    def token(self, which: str) -> int:
        return self.L.oracle_token(self.m, which.encode())

    def mel(self, pcm: np.ndarray):
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        org = C.c_int()
        n_len = self.L.oracle_mel(self.m, self.s, _fp(pcm), len(pcm), C.byref(org))
        out = np.empty((self.n_mels, n_len), np.float32)
        self.L.oracle_state_mel(self.s, _fp(out))
        return out, org.value

    def set_mel(self, mel: np.ndarray):
        mel = np.ascontiguousarray(mel, dtype=np.float32)
        self.L.oracle_set_mel(self.m, self.s, _fp(mel), mel.shape[1])

    def encode(self, seek: int = 0) -> np.ndarray:
        out = np.empty((self.n_audio_ctx, self.d), np.float32)
        self.L.oracle_encode(self.m, self.s, seek, _fp(out))
        return out

    def cross_kv(self, layer: int):
        k = np.empty((self.n_audio_ctx, self.d), np.float32)
        v = np.empty_like(k)
        self.L.oracle_cross_kv(self.m, self.s, layer, _fp(k), _fp(v))
        return k, v

    def kv_clear(self):
        self.L.oracle_kv_clear(self.s)

    def decode(self, tokens, n_past: int) -> np.ndarray:
        t = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.empty((len(t), self.n_vocab), np.float32)
        self.L.oracle_decode(self.m, self.s, _ip(t), len(t), n_past, _fp(out))
        return out

    def tokenize(self, text: str):
        buf = np.empty(4096, np.int32)
        n = self.L.oracle_tokenize(self.m, text.encode(), _ip(buf), len(buf))
        return buf[:n].tolist()

    def token_str(self, i: int) -> bytes:
        return self.L.oracle_token_str(self.m, i)

    def full(self, pcm: np.ndarray, params: OracleParams) -> dict:
        pcm = np.ascontiguousarray(pcm, dtype=np.float32)
        rc = self.L.oracle_full(self.m, self.s, C.byref(params), _fp(pcm), len(pcm))
        segs = []
        for i in range(self.L.oracle_n_segments(self.s)):
            t0, t1 = C.c_int64(), C.c_int64()
            self.L.oracle_segment_t(self.s, i, C.byref(t0), C.byref(t1))
            toks = [self.L.oracle_segment_token(self.s, i, j) for j in range(self.L.oracle_segment_n_tokens(self.s, i))]
            segs.append(dict(t0=t0.value, t1=t1.value, text=self.L.oracle_segment_text(self.s, i), tokens=toks,
                             seek=self.L.oracle_segment_seek(self.s, i)))
        n = self.L.oracle_n_steps(self.s)
        margins = np.empty(n, np.float32)
        self.L.oracle_step_margins(self.s, _fp(margins))
        step_tok = np.empty(max(1, n), np.int32)
        step_seek = np.empty(max(1, n), np.int32)
        self.L.oracle_step_tokens(self.s, _ip(step_tok), _ip(step_seek))
        seq = (C.c_int * 4096)()
        n_seq = min(4096, self.L.oracle_decoder_tokens(self.s, seq, 4096))
        nd = self.L.oracle_n_decisions(self.s)
        dec = (Decision * max(1, nd))()
        self.L.oracle_decisions(self.s, C.cast(dec, C.c_void_p))
        out = dict(rc=rc, segments=segs, lang=self.L.oracle_lang(self.s),
                   no_speech_prob=self.L.oracle_no_speech(self.s), margins=margins, seq=list(seq[:n_seq]),
                   step_tokens=step_tok[:n].tolist(), step_seeks=step_seek[:n].tolist(),
                   decisions=decisions_to_dicts(dec[:nd]))
        if params.fixed_tokens > 0:
            # the raw logits of every step ([steps][V]): what a teacher-forced pass along the greedy
            # sequence computes (same prompt, same cross K/V), recorded instead of decoded a second time
            rows = self.L.oracle_step_logits(self.m, self.s, None, 0)
            lg = np.empty((rows, self.n_vocab), np.float32)
            self.L.oracle_step_logits(self.m, self.s, _fp(lg), lg.size)
            out["step_logits"] = lg
        return out


# ---- one oracle per model file and one result per (model, input, params) for the whole pytest session ----
# (the full-depth oracle runs ~13 s per large-v3 encoder pass; test modules that
# compare against the same oracle result share it instead of recomputing it)
_SHARED = {}
_FULL = {}


def shared_oracle(path: str, mode: int = 1, n_threads: int = 16) -> "Oracle":
    key = (path, mode)
    if key not in _SHARED:
        _SHARED[key] = Oracle(path, mode=mode, n_threads=n_threads)
    return _SHARED[key]


def params_key(p: OracleParams) -> tuple:
    return tuple(getattr(p, f) for f, _ in OracleParams._fields_)


def cached_full(path: str, pcm_key, pcm_fn, params: OracleParams, mode: int = 1) -> dict:
    """Oracle.full on a fresh state (whisper.rs:83-85: a new state per call), computed once per session
    for (model file, pcm_key, params); pcm_fn() makes the input on a miss."""
    key = (path, mode, pcm_key, params_key(params))
    if key not in _FULL:
        o = shared_oracle(path, mode)
        o.new_state()
        _FULL[key] = o.full(pcm_fn(), params)
    return _FULL[key]


# ---- audio.rs restatement (oracle/oracle_audio.cpp) -------------------------------------------------
def calculate_rms(x) -> float:
    x = np.ascontiguousarray(x, dtype=np.float32)
    return float(lib().oracle_calculate_rms(_fp(x), len(x)))


def estimate_noise_floor(x, sr: int) -> float:
    x = np.ascontiguousarray(x, dtype=np.float32)
    return float(lib().oracle_estimate_noise_floor(_fp(x), len(x), sr))


def find_silence_boundaries(x, sr: int) -> list:
    x = np.ascontiguousarray(x, dtype=np.float32)
    cap = len(x) // max(1, sr) + 2
    out = np.zeros(cap, np.int32)
    n = lib().oracle_find_silence_boundaries(_fp(x), len(x), sr, _ip(out), cap)
    return out[:n].tolist()


def split_at_silences(n: int, bounds, sr: int) -> list:
    b = np.ascontiguousarray(bounds, dtype=np.int32)
    cap = len(b) + 2
    s, e = np.zeros(cap, np.int32), np.zeros(cap, np.int32)
    k = lib().oracle_split_at_silences(n, _ip(b), len(b), sr, _ip(s), _ip(e), cap)
    return list(zip(s[:k].tolist(), e[:k].tolist()))


def resample(x, rate_in: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    cap = int(len(x) * 16000 / rate_in) + 2048
    out = np.zeros(max(cap, 1), np.float32)
    n = lib().oracle_resample(_fp(x), len(x), rate_in, _fp(out), cap)
    return out[:n].copy()


# ---- audio.rs:29-241 AudioBuffer, restated in numpy (test infrastructure) -------------------------
# Independent of the product's C++ (nobs-whisper_amd/host/audio_buffer.cpp): every f32 sum is a
# float32 np.cumsum (numpy accumulates sequentially, as Rust's Iterator::sum), every product and
# constant float32.
_F = np.float32


def rms_f32(x) -> np.float32:
    """audio.rs:364-370"""
    x = np.asarray(x, dtype=np.float32)
    if len(x) == 0:
        return _F(0.0)
    s = np.cumsum(x * x, dtype=np.float32)[-1]
    return np.sqrt(_F(s) / _F(len(x)))


class AudioBufferRef:
    SILENCE = _F(0.01)
    MIN_THR = _F(0.01) * _F(0.5)
    ONE_MINUS = _F(1.0) - _F(0.95)

    def __init__(self, sample_rate: int = 48000):
        self.sr = sample_rate
        self._parts, self._n = [], 0
        self.last_speech_pos = 0
        self.noise_floor = _F(0.01)
        self.noise_floor_frames = 0
        self.overlap = np.zeros(0, np.float32)

    @property
    def samples(self):
        if len(self._parts) != 1:
            self._parts = [np.concatenate(self._parts) if self._parts else np.zeros(0, np.float32)]
        return self._parts[0]

    @samples.setter
    def samples(self, v):
        self._parts, self._n = [v], len(v)

    def push_samples(self, x):
        x = np.asarray(x, dtype=np.float32)
        start = self._n
        self._parts.append(x)
        self._n += len(x)
        w = self.sr // 50
        for i, off in enumerate(range(0, len(x), w)):
            rms = rms_f32(x[off:off + w])
            if rms < self.noise_floor * _F(0.5) and self.noise_floor_frames < 100:
                self.noise_floor = _F(self.noise_floor * _F(0.95)) + _F(rms * self.ONE_MINUS)
                self.noise_floor_frames += 1
            thr = max(_F(self.noise_floor * _F(3.0)), self.MIN_THR)
            if rms >= thr:
                self.last_speech_pos = start + (i + 1) * w

    def take(self):
        self.last_speech_pos = 0
        self.overlap = np.zeros(0, np.float32)
        out, self.samples = self.samples, np.zeros(0, np.float32)
        return out

    def has_silence_boundary(self) -> bool:
        if self._n == 0 or self.last_speech_pos == 0:
            return False
        return max(0, self._n - self.last_speech_pos) >= self.sr * 700 // 1000

    def _emit(self, split):
        ov = self.sr * 200 // 1000
        chunk = np.concatenate([self.overlap, self.samples[:split]])
        self.overlap = self.samples[max(0, split - ov):split].copy()
        self.samples = self.samples[split:].copy()
        return chunk

    def take_chunk_at_silence(self):
        if not self.has_silence_boundary() or self.last_speech_pos < self.sr // 2:
            return None
        s0 = self.last_speech_pos
        chunk = self._emit(s0 + (self._n - s0) // 2)
        self.last_speech_pos = 0
        return chunk

    def take_forced_chunk(self):
        n = self._n
        if n <= self.sr * 25:
            return None
        w = self.sr // 50
        start = max(0, n - self.sr * 5)
        q_pos, q_rms = start, np.finfo(np.float32).max
        pos = start
        while pos + w <= n:
            r = rms_f32(self.samples[pos:pos + w])
            if r < q_rms:
                q_rms, q_pos = r, pos
            pos += w
        split = min(q_pos + w // 2, n)
        if split < self.sr // 2:
            return None
        chunk = self._emit(split)
        self.last_speech_pos = self.last_speech_pos - split if self.last_speech_pos > split else 0
        return chunk
