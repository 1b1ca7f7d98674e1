"""GPU experiment: does a second batch's encoder overlap the first batch's decode on one GPU?

Two whisper_states on one context (each has its own HIP streams), 128 x 30 s large-v3 chunks in HBM,
fixed-work mode (128 tokens). (a) two full_batch calls back to back on one state; (b) two calls from
two host threads (ctypes releases the GIL), the second started `delay` seconds after the first, so its
encoder (~0.33 s) runs beside the first call's decode (~0.86 s). Prints wall times and the implied
throughput of each schedule.
"""
import ctypes as C
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import bench  # noqa: E402

wrs = bench.load_wrs()
B = int(os.environ.get("OV_BATCH", "128"))
model_dir = os.environ.get("NW_MODEL_DIR", "/tmp/nw_models")
os.makedirs(model_dir, exist_ok=True)
path = os.path.join(model_dir, "large-v3+conf_s0.bin")
bench.ensure_model(path, "large-v3+conf")
ctx = wrs.WhisperContext(path, dtype=wrs.BF16)
L = wrs.lib()
import numpy as np  # noqa: E402
from make_model import synthetic_pcm  # noqa: E402
n = 16000 * 30
buf = L.whisper_mi355x_dev_alloc(ctx.ptr, B * n * 4)
host = np.empty(n, np.float32)
for i in range(B):
    host[:] = synthetic_pcm(i)
    L.whisper_mi355x_memcpy(ctx.ptr, C.c_void_p(buf + i * n * 4), host.ctypes.data, n * 4, 1)
jobs = [(buf + i * n * 4, n) for i in range(B)]
params = wrs.reference_full_params("en")
s1, s2 = ctx.create_state(), ctx.create_state()


def run(st):
    assert st.full_batch(params, jobs, on_device=True, fixed_tokens=128) == 0


for st in (s1, s2):  # warm-up: workspaces, decode graphs
    run(st)
t = time.perf_counter()
run(s1)
run(s1)
seq = time.perf_counter() - t
print(f"sequential 2 batches: {seq:.3f} s  ({2 * B * 30 / seq:.0f} audio-s/s); phases of the last: {s1.phase_ms()}", flush=True)
for delay in [float(x) for x in os.environ.get("OV_DELAYS", "0,0.2,0.35,0.5").split(",")]:
    t = time.perf_counter()
    th = threading.Thread(target=run, args=(s2,))
    th_started = [0.0]

    def second():
        time.sleep(delay)
        th_started[0] = time.perf_counter() - t
        run(s2)
    th = threading.Thread(target=second)
    th.start()
    run(s1)
    t1 = time.perf_counter() - t
    th.join()
    tot = time.perf_counter() - t
    print(f"concurrent, second start {delay:.2f} s: first done {t1:.3f} s, both {tot:.3f} s "
          f"({2 * B * 30 / tot:.0f} audio-s/s vs {2 * B * 30 / seq:.0f} sequential); s1 {s1.phase_ms()} s2 {s2.phase_ms()}",
          flush=True)
