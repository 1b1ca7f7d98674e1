"""The C-ABI boundary without a GPU: the library loads, exports every symbol include/*.h declares,
and the ctypes mirror of whisper_full_params agrees with the C layout field by field."""
import ctypes as C
import os
import re
import subprocess

from conftest import ROOT

LIB = os.path.join(ROOT, "nobs-whisper_amd", "lib", "libwhisper_mi355x.so")
HDRS = [os.path.join(ROOT, "include", h) for h in ("whisper.h", "whisper_mi355x.h")]


def declared_symbols():
    names = set()
    for h in HDRS:
        text = "\n".join(ln for ln in open(h).read().splitlines() if not ln.startswith("#define"))
        for m in re.finditer(r"WHISPER_API\s+[^;(]*?\b(\w+)\s*\(", text):
            names.add(m.group(1))
    return names


def test_library_loads():
    C.CDLL(LIB)


def test_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    declared = declared_symbols()
    assert len(declared) > 110
    missing = sorted(declared - exported)
    assert not missing, missing


def test_full_params_layout_matches_ctypes(wrs):
    L = wrs.lib()
    out = (C.c_size_t * 8)()
    assert L.whisper_mi355x_abi_layout(out) == 8
    FP = wrs.FullParams
    assert out[0] == C.sizeof(FP)
    assert out[1] == C.sizeof(wrs.WhisperContextParams)
    assert out[2] == C.sizeof(wrs.TokenData)
    assert out[3] == FP.initial_prompt.offset
    assert out[4] == FP.language.offset
    assert out[5] == FP.greedy.offset
    assert out[6] == FP.new_segment_callback.offset
    assert out[7] == FP.vad_params.offset


def test_default_params_match_whisper_cpp(wrs):
    """whisper_full_default_params(GREEDY) values the reference relies on (whisper.rs:88-124 only
    overrides some of them)."""
    p = wrs.lib().whisper_full_default_params(wrs.GREEDY)
    assert p.strategy == 0 and p.greedy.best_of == 5 and p.n_max_text_ctx == 16384
    assert p.no_context is True and p.suppress_blank is True and p.language == b"en"
    assert abs(p.temperature) == 0 and abs(p.temperature_inc - 0.2) < 1e-7 and abs(p.max_initial_ts - 1.0) < 1e-7
    assert abs(p.entropy_thold - 2.4) < 1e-6 and abs(p.logprob_thold + 1.0) < 1e-7 and abs(p.no_speech_thold - 0.6) < 1e-7
    cp = wrs.lib().whisper_context_default_params()
    assert cp.use_gpu is True and cp.gpu_device == 0


def test_lang_table(wrs):
    L = wrs.lib()
    assert L.whisper_lang_id(b"en") == 0 and L.whisper_lang_id(b"ko") == 5 and L.whisper_lang_id(b"yue") == 99
    assert L.whisper_lang_str(7) == b"ja"
    assert L.whisper_lang_id(b"klingon") == -1
