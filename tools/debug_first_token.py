"""GPU debug: decoder logits and first greedy token, oracle vs HIP path (micro + tiny)."""
import ctypes as C
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_whisper_rs, model_path
from make_model import synthetic_pcm
from oracle_py import Oracle, reference_params

wrs = load_whisper_rs()
L = wrs.lib()
for shape in ("micro", "tiny"):
    path = model_path(shape)
    pcm = synthetic_pcm(0)
    o = Oracle(path, mode=1)
    o.mel(pcm); o.encode(0); o.kv_clear()
    sot = o.token("sot")
    prompt = [sot, sot + 1, o.token("transcribe")]
    ref = o.decode(prompt, 0)[-1]
    ctx = wrs.WhisperContext(path, dtype=wrs.F16)
    st = ctx.create_state()
    a = np.ascontiguousarray(pcm)
    L.whisper_pcm_to_mel_with_state(ctx.ptr, st.ptr, a.ctypes.data_as(C.POINTER(C.c_float)), len(a), 1)
    L.whisper_encode_with_state(ctx.ptr, st.ptr, 0, 1)
    arr = (C.c_int * 3)(*prompt)
    L.whisper_decode_with_state(ctx.ptr, st.ptr, arr, 3, 0, 1)
    V = L.whisper_n_vocab(ctx.ptr)
    g = np.ctypeslib.as_array(L.whisper_get_logits_from_state(st.ptr), shape=(3 * V,)).reshape(3, V)[-1].copy()
    print(shape, "logits maxabs", float(np.abs(g - ref).max()), "argmax", int(g.argmax()), int(ref.argmax()))
    st2 = ctx.create_state()
    rc = st2.full_batch(wrs.reference_full_params("en"), [pcm], fixed_tokens=4)
    segs = st2.batch_segments(0)
    r = o.full(pcm, reference_params("en", fixed_tokens=4))
    print(shape, "fixed4 gpu", [[t[0] for t in s.tokens] for s in segs], "oracle", [s["tokens"] for s in r["segments"]])
    st3 = ctx.create_state()
    st3.full(wrs.reference_full_params("en"), pcm)
    r = o.full(pcm, reference_params("en"))
    print(shape, "full gpu", [[t[0] for t in s.tokens][:6] for s in st3.segments()][:3], "oracle", [s["tokens"][:6] for s in r["segments"]][:3])
    print(shape, "oracle margins head", r["margins"][:5])
