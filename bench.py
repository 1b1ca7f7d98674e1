#!/usr/bin/env python3
"""Throughput benchmark: audio-seconds/s of greedy Whisper transcription on MI355X.

Metric (BASELINE.json): "audio-sec/s (RTF^-1) large-v3 greedy, batch 128; 1/2/4/8 MI355X".
One step = whisper_mi355x_full_batch over this rank's share of a global batch of 30 s chunks (PCM
already resident in HBM): log-mel -> encoder -> cross attention -> prefill -> fixed-work greedy
decode of --tokens tokens per chunk (EOT suppressed, no fallback: SURVEY.md §8d's reproducible-work
mode for random weights) -> logits processing -> segments.

Multi-GPU (BASELINE config 4): strong scaling of --global-batch chunks (default 128):
rank r transcribes chunks [r*ceil(B/n), min(B, (r+1)*ceil(B/n))); ranks share no data-path
collective; rank 0 loads the weights and broadcasts the packed arena once over RCCL/xGMI (outside
the timed region, reported as weight_broadcast_s). `--gpus N` without a torch.distributed launcher
spawns the N rank processes itself (before any GPU call); under torchrun it reads RANK/WORLD_SIZE.

Model weights are a seeded synthetic GGML file of the named architecture (no checkpoints offline);
audio is synthetic (tools/make_model.synthetic_pcm, seed 1234 + global chunk index).

Run:  python bench.py [--gpus N --steps K --warmup W]
      torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "audio-sec/s (RTF⁻¹) large-v3 greedy, batch 128; 1/2/4/8 MI355X"
K_NAMES = ["gemm_encoder", "attn_encoder", "attn_cross_decode", "attn_self_decode", "gemm_decode", "logits", "mel",
           "pdec_step"]
K_BOUND = ["mfma", "mfma", "hbm", "hbm", "hbm", "hbm", "hbm", "hbm"]
SINGLE_KERNEL = [1, 2, 3, 5, 6, 7]  # classes that are one kernel each (attention, logits, mel, persistent step)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_PEAK_TFS = 2500.0       # dense bf16/f16 MFMA peak (no sparsity)
FP8_PEAK_TFS = 5000.0        # dense fp8 MFMA peak
# PMC traffic pass of the roofline kernel (tools/pmc.sh -> tools/pmc_traffic.py), chosen by name
PMC_TRAFFIC_FILE = "r06_pmc_traffic.json"
KT_LAYER_STRIDE = 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_wrs():
    import importlib.util
    spec = importlib.util.spec_from_file_location("whisper_rs", os.path.join(ROOT, "nobs-whisper_amd", "whisper_rs.py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules["whisper_rs"] = m
    spec.loader.exec_module(m)
    return m


def ensure_model(path: str, shape: str):
    from make_model import write_model
    if not os.path.exists(path):
        t = time.time()
        last = [t]

        def progress(name):  # a quantized large-v3 takes minutes to write: say that it moves
            if time.time() - last[0] > 20:
                last[0] = time.time()
                log(f"[bench] writing {shape}: {name} ({time.time() - t:.0f}s)")

        write_model(path, shape, 0, progress=progress)
        log(f"[bench] wrote synthetic {shape} model to {path} in {time.time() - t:.1f}s")


def cgroup_cpus():
    """CPUs this job may use under its cgroup quota (cgroup v2 cpu.max "quota period", v1 cfs files),
    or None when no quota caps it."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            return dict(cpu_max=f"{q} {p}", cpus=int(q) / int(p))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            p = int(f.read())
        if q > 0:
            return dict(cpu_max=f"{q} {p}", cpus=q / p)
    except (OSError, ValueError):
        pass
    return None


def host_cpu() -> dict:
    """The node's CPU (lscpu model name, logical CPUs) and every CPU this job may use: the scheduler
    affinity set, capped by the cgroup's CPU quota when one is set (cpu.max)."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
    except Exception:
        pass
    aff = len(os.sched_getaffinity(0))
    cg = cgroup_cpus()
    if cg is not None:
        usable = max(1, min(aff, int(cg["cpus"])))
    else:  # no quota visible: the box's declared share (it sets OMP_NUM_THREADS to the job's CPUs), else affinity
        usable = min(aff, int(os.environ.get("OMP_NUM_THREADS") or aff))
    return dict(model=model, logical_cpus=os.cpu_count(), affinity=aff,
                cgroup_cpu_max=cg["cpu_max"] if cg else None, usable=usable,
                omp_num_threads_env=os.environ.get("OMP_NUM_THREADS"))


def cpu_baseline(model_path: str, threads: int, n_tokens: int, n_sample_tokens: int = 0) -> dict:
    """The CPU oracle (restated whisper.cpp algorithm, C++/OpenMP) on a bounded sample of the same
    workload: 1 chunk = mel + encoder + cross-KV + 3-token prefill + n_sample_tokens decode steps
    (default: all n_tokens of the fixed-work mode, so nothing is extrapolated; large-v3 on 16 threads
    is ~13 s of encoder + ~4 s of decode)."""
    n_sample_tokens = n_sample_tokens or n_tokens
    from make_model import synthetic_pcm
    from oracle_py import Oracle
    o = Oracle(model_path, mode=1, n_threads=threads)
    pcm = synthetic_pcm(0)
    t0 = time.time()
    o.mel(pcm)
    t1 = time.time()
    o.encode(0)
    t2 = time.time()
    o.kv_clear()
    sot = o.token("sot")
    prompt = [sot, sot + 1, o.token("transcribe")]
    lg = o.decode(prompt, 0)
    t3 = time.time()
    tok = int(lg[-1].argmax())
    for i in range(n_sample_tokens):
        lg = o.decode([tok], len(prompt) + i)
        tok = int(lg[-1].argmax())
    t4 = time.time()
    o.close()
    per_step = (t4 - t3) / n_sample_tokens
    chunk_s = (t1 - t0) + (t2 - t1) + (t3 - t2) + n_tokens * per_step
    cpu = host_cpu()
    extra = "" if n_sample_tokens == n_tokens else f", extrapolated to {n_tokens} steps/chunk"
    return dict(value=round(30.0 / chunk_s, 3), unit="audio-sec/s", cores=threads, kind="port",
                host_cpu=cpu,
                sample=(f"1 x 30 s chunk: mel {t1 - t0:.2f}s + encoder/cross-KV {t2 - t1:.2f}s + prefill {t3 - t2:.2f}s "
                        f"+ {n_sample_tokens} decode steps ({per_step * 1e3:.0f} ms/step) measured{extra}; "
                        f"oracle/ = restated whisper.cpp CPU algorithm (not whisper.cpp), "
                        f"{threads} OpenMP threads = every CPU this job may use (affinity {cpu['affinity']}, "
                        f"cgroup cpu.max {cpu['cgroup_cpu_max']}) of a {cpu['logical_cpus']}-CPU {cpu['model']} host"))


# kernel symbol of each class in the rocprofv3 PMC output (tools/pmc.sh -> tools/pmc_traffic.py), per
# cross-attention form for the decode-step class: straight from the encoder output, or the cached K/V
K_SYMBOL = {("gemm_encoder", None): r"gemm8p_kernel", ("attn_encoder", None): r"attn_enc2_kernel",
            ("attn_cross_decode", True): r"xattn_step_kernel",
            ("attn_cross_decode", False): r"attn_cross_step_(wide_)?kernel", ("pdec_step", None): r"pdec_kernel"}


def cross_step_grid(direct: bool, nb: int, heads: int, wide_max: int = 4) -> int:
    """Threads per decode-step launch of the cross-attention kernel (the PMC pass is keyed by it):
    direct form, xattn_step_kernel: xattn_splits(nb) x nb workgroups of 512 threads; cache form,
    attn_cross_step_kernel: nb x H workgroups of 256 threads, or 1024 (the wide kernel) at <= 4 clips."""
    if direct:
        return max(1, min(16, -(-256 // nb))) * nb * 512
    return nb * heads * (1024 if nb <= wide_max else 256)


def pmc_traffic(kernel_class: str, direct: bool | None, grid_threads: int | None, sym_re: str = ""):
    """Launch-weighted HBM bytes per launch (FETCH_SIZE doubled per the gfx950 correction, +
    WRITE_SIZE) of the kernel this class launched in the timed steps, from profiles/PMC_TRAFFIC_FILE:
    matched by kernel symbol (and cross form) AND grid size (and sym_re: the persistent step's width and
    compute type, whose grid is the same for every model), or None when that pass did not profile this
    exact launch shape."""
    import re
    pat = K_SYMBOL.get((kernel_class, direct if kernel_class == "attn_cross_decode" else None))
    path = os.path.join(ROOT, "profiles", PMC_TRAFFIC_FILE)
    if not pat or grid_threads is None or not os.path.exists(path):
        return None, None
    with open(path) as f:
        data = json.load(f)
    n = tb = 0.0
    for sym, v in data.items():
        name, _, grid = sym.partition("@grid=")
        if re.search(pat, name) and grid == str(grid_threads) and re.search(sym_re, name):
            n += v["launches"]
            tb += v["traffic_bytes"] * v["launches"]
    return (tb / n if n else None), PMC_TRAFFIC_FILE


def rank_chunk_ids(rank: int, world: int, global_batch: int) -> list[int]:
    """Strong-scaling shard: contiguous blocks of ceil(B/n) chunks per rank; the last
    rank may get fewer. Independent 30 s chunks: no data-path exchange between ranks."""
    per = -(-global_batch // world)
    return list(range(rank * per, min(global_batch, (rank + 1) * per)))


def max_over_ranks(x: float, dist, device: str) -> float:
    """The timed region's wall time is the slowest rank's (contract: max over ranks)."""
    if dist is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def phase_work(shape: str, n_chunks: int, tokens: int, prompt_len: int, direct: bool) -> dict:
    """Algorithmic work of one step: encoder FLOPs (conv stem + layers incl.
    attention) and the decode steps' HBM bytes (decoder weights + token embedding once per step,
    the encoder output E once per clip and layer (direct cross attention; the K + V cache when not
    direct), the self-KV prefix)."""
    from make_model import SHAPES as S
    V, nm, d, h, Le, Ld = S[shape]
    T = 1500
    conv = 2.0 * 2 * T * 3 * nm * d + 2.0 * T * 3 * d * d
    layer = 2.0 * T * d * 12 * d + 4.0 * T * T * d
    enc_flops = n_chunks * (conv + Le * layer)
    # fp8 mode (--dtype fp8): the QKV, FC1 and FC2 GEMMs (11 d^2 per token) run on the fp8 pipe
    enc_flops_fp8 = n_chunks * Le * 2.0 * T * d * 11 * d
    w_bytes = (Ld * 16 * d * d + V * d) * 2.0
    xa_bytes = n_chunks * Ld * T * d * 2.0 * (1 if direct else 2)
    avg_pos = prompt_len + tokens / 2.0
    self_bytes = n_chunks * Ld * 2 * avg_pos * d * 2.0
    return dict(enc_flops=enc_flops, enc_flops_fp8=enc_flops_fp8, dec_bytes_per_step=w_bytes + xa_bytes + self_bytes,
                dec_weight_bytes=w_bytes, dec_cross_bytes=xa_bytes, dec_self_bytes=self_bytes)


def spawn_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N rank processes (one per GPU) with the torch.distributed
    env, before this process touches the GPU; return the worst exit code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def plan(rank: int, world: int, args) -> None:
    """--plan: the multi-rank layout without a GPU (tests/test_dist.py): every rank joins a gloo
    group, computes its shard and a rank-dependent "elapsed", and rank 0 prints the max over ranks
    and the gathered shard map as one JSON line."""
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    ids = rank_chunk_ids(rank, world, args.global_batch)
    t = max_over_ranks(0.25 * (rank + 1), dist, "cpu")
    shards = [ids]
    if dist is not None:
        shards = [None] * world
        dist.all_gather_object(shards, ids)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "max_elapsed": t, "shards": shards}), flush=True)


def bench_frontend(wrs, ctx, buf, nb: int, n: int, reps: int = 5) -> dict:
    """The reference's audio front-end (src-tauri/src/audio.rs) on this rank's chunks, device-resident:
    find_silence_boundaries over the nb 16 kHz chunks (HBM-bound: 4 B per sample), and
    resample_chunk of nb 30 s 48 kHz captures (f32 VALU-bound: 4 * fsi * fso FLOP per 171-sample
    output block). Host wall clock around the synchronous C-ABI calls, best of `reps`."""
    import numpy as np
    L = wrs.lib()
    dev = ctx.gpu_device
    ptrs = (C.c_void_p * nb)(*[buf + i * n * 4 for i in range(nb)])
    ns = (C.c_int * nb)(*([n] * nb))
    cap = n // 16000 + 2
    counts = np.zeros(nb, np.int32)
    bnd = np.zeros((nb, cap), np.int32)
    ip = C.POINTER(C.c_int)

    def vad():
        assert L.whisper_mi355x_find_silence_boundaries(dev, ptrs, ns, nb, 16000, True, counts.ctypes.data_as(ip),
                                                        bnd.ctypes.data_as(ip), cap, None, None, 0) == 0
    vad()
    t_vad = min(_wall(vad) for _ in range(reps))
    rate, n48 = 48000, 48000 * 30
    n16 = L.whisper_mi355x_resample_len(n48, rate)
    src = L.whisper_mi355x_dev_alloc(ctx.ptr, nb * n48 * 4)
    dst = L.whisper_mi355x_dev_alloc(ctx.ptr, nb * n16 * 4)
    assert src and dst
    from make_model import synthetic_pcm
    host = synthetic_pcm(0, seconds=30.0, sr=rate).astype(np.float32)
    for i in range(nb):
        L.whisper_mi355x_memcpy(ctx.ptr, C.c_void_p(src + i * n48 * 4), host.ctypes.data, n48 * 4, 1)
    iptr = (C.c_void_p * nb)(*[src + i * n48 * 4 for i in range(nb)])
    optr = (C.c_void_p * nb)(*[dst + i * n16 * 4 for i in range(nb)])
    nin = (C.c_int * nb)(*([n48] * nb))

    def rs():
        assert L.whisper_mi355x_resample_chunk(dev, iptr, nin, nb, rate, True, optr) == 0
    rs()
    t_rs = min(_wall(rs) for _ in range(reps))
    L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(src))
    L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(dst))
    fsi, fso = C.c_int(), C.c_int()
    L.whisper_mi355x_resample_operator(rate, C.byref(fsi), C.byref(fso), None, 0)
    flops = nb * (-(-n16 // fso.value)) * 4.0 * fsi.value * fso.value
    vad_bytes = nb * n * 4.0
    return {
        "clips": nb, "vad_boundaries_per_clip": float(counts.mean()),
        "find_silence_boundaries": dict(ms=round(t_vad * 1e3, 3), audio_s_per_s=round(30.0 * nb / t_vad, 1),
                                        gb_s=round(vad_bytes / t_vad / 1e9, 1),
                                        hbm_frac=round(vad_bytes / t_vad / 1e9 / HBM_PEAK_GBS, 4)),
        "resample_48k_to_16k": dict(ms=round(t_rs * 1e3, 3), audio_s_per_s=round(30.0 * nb / t_rs, 1),
                                    tflop_s=round(flops / t_rs / 1e12, 2),
                                    note="f32 VALU operator product (rubato FftFixedIn folded); wall clock "
                                         "around the synchronous call incl. pointer-table uploads"),
    }


def app_pattern(wrs, model_dir: str, shape: str, dtype: str, calls: int) -> dict:
    """The reference app's own call pattern, per call (src-tauri/src/state.rs:147 streaming worker ->
    whisper.rs:66-148 through the C++ mirror of WhisperEngine, host/whisper_engine.cpp): a fresh
    whisper_state per call (whisper.rs:83-85), one <= 25.2 s chunk (audio.rs:11,15: forced cut at 25 s +
    200 ms overlap), language "auto" (config.rs:49), initial prompt = the default vocabulary + the
    previous chunk's text (config.rs:40-42, whisper.rs:98-105, state.rs:144-151), segments joined and
    filtered. Latency per call = host wall clock around transcribe (PCM on the host, results on the
    host). Measured with the context's state pool (default: a released state keeps its workspace and
    decode graphs for the next call) and without it (WHISPER_MI355X_STATE_POOL=0: every call allocates
    its workspace and captures its decode graphs, as a plain whisper.cpp state would). Every call's decoded
    tokens (all decode steps of all attempts, whisper_mi355x_decoded_tokens_total around the call) are
    reported beside its latency, so calls that decode more tokens are not mistaken for slower ones."""
    import numpy as np
    from make_model import synthetic_pcm
    path = os.path.join(model_dir, f"{shape}_s0.bin")
    ensure_model(path, shape)
    os.environ["WHISPER_MI355X_DTYPE"] = dtype
    chunks = [synthetic_pcm(100 + k, seconds=25.2) for k in range(calls)]
    out = {"model": shape, "dtype": dtype, "chunk_s": 25.2, "calls": calls}
    for label, pool in (("state_pool", "2"), ("no_pool", "0")):
        os.environ["WHISPER_MI355X_STATE_POOL"] = pool
        eng = wrs.WhisperEngine()
        assert eng.load_model(path) == 0
        last, lat, toks, chars = None, [], [], 0
        L = wrs.lib()
        for x in chunks:
            k0 = L.whisper_mi355x_decoded_tokens_total()
            t = time.perf_counter()
            rc, text = eng.transcribe(x, None, wrs.DEFAULT_VOCABULARY, last)
            lat.append(time.perf_counter() - t)
            toks.append(L.whisper_mi355x_decoded_tokens_total() - k0)
            assert rc == 0, rc
            last = text or None
            chars += len(text or "")
        del eng
        steady = sorted(lat[1:]) or lat
        per_tok = sorted(1e3 * a / max(1, b) for a, b in list(zip(lat, toks))[1:]) or [1e3 * lat[0] / max(1, toks[0])]
        out[label] = dict(first_call_ms=round(lat[0] * 1e3, 1), median_ms=round(1e3 * steady[len(steady) // 2], 1),
                          min_ms=round(1e3 * min(steady), 1),
                          rtf_inverse_median=round(25.2 / steady[len(steady) // 2], 1),
                          decoded_tokens_per_call=toks, ms_per_decoded_token_median=round(per_tok[len(per_tok) // 2], 3),
                          ms_per_call=[round(1e3 * a, 1) for a in lat])
    out["text_chars_total"] = chars
    os.environ.pop("WHISPER_MI355X_STATE_POOL", None)
    os.environ.pop("WHISPER_MI355X_DTYPE", None)
    return out


def _wall(fn) -> float:
    t = time.perf_counter()
    fn()
    return time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="large-v3")
    ap.add_argument("--global-batch", type=int, default=128, help="30 s chunks per step over all GPUs (strong scaling)")
    ap.add_argument("--batch", type=int, default=0, help="weak scaling instead: chunks per GPU (0 = off)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f16", "fp8"],
                    help="fp8: bf16 with the encoder QKV/FC1/FC2 GEMMs on e4m3 weights + activations")
    ap.add_argument("--tokens", type=int, default=128, help="decode tokens per chunk (fixed-work mode)")
    ap.add_argument("--variants", type=int, default=1,
                    help="also time the reference's prompted (default vocabulary) and auto-language workloads")
    ap.add_argument("--variant-steps", type=int, default=3)
    ap.add_argument("--inflight-line", type=int, default=1,
                    help="with --variants: also a serving line with two batches in flight (two states)")
    ap.add_argument("--f16-line", type=int, default=1,
                    help="with --dtype bf16: also time the same config with f16 weights (the path exact against the oracle up to its near ties)")
    ap.add_argument("--fallback-line", type=int, default=0,
                    help="also time the reference's verbatim FullParams with temperature fallback (slow on "
                         "untrained weights: most windows fall back to sampled re-decodes)")
    ap.add_argument("--frontend", type=int, default=1,
                    help="also time the GPU audio front-end (audio.rs VAD chunking + 48 kHz -> 16 kHz resampler)")
    ap.add_argument("--app-pattern", type=int, default=1,
                    help="also time the app's per-call pattern (fresh state per 25 s chunk, whisper.rs:66-148) "
                         "on base f16 and this model in its dtype (rank 0)")
    ap.add_argument("--app-calls", type=int, default=6)
    ap.add_argument("--quant", default="none", choices=["none", "q4_0", "q4_1", "q5_0", "q5_1", "q8_0"],
                    help="GGML block-quantized model file (the app's catalog ships large-v3-q5_0): blocks stay "
                         "quantized in HBM, dequantized inside the GEMMs")
    ap.add_argument("--weights", default="conf", choices=["conf", "plain"],
                    help="synthetic weight init: conf = a decoder as peaked as a trained one (tools/make_model.py "
                         "+conf), so real greedy termination happens; plain = i.i.d. random")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU this job may use (affinity, capped by the cgroup cpu.max quota)")
    ap.add_argument("--model-dir", default=os.environ.get("NW_MODEL_DIR", "/tmp/nw_models"))
    ap.add_argument("--plan", action="store_true",
                    help="CPU dry run of the rank layout: gloo group, shard map and max-over-ranks, no GPU")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plan:
        return plan(rank, world, args)
    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    def barrier():
        if dist is not None:
            dist.barrier()

    wrs = load_wrs()
    os.makedirs(args.model_dir, exist_ok=True)
    shape = args.model + ("+conf" if args.weights == "conf" else "") + ("" if args.quant == "none" else "+" + args.quant)
    model_path = os.path.join(args.model_dir, f"{shape}_s0.bin")
    if local_rank == 0:
        ensure_model(model_path, shape)
    barrier()

    # ---- context: rank 0 loads, the others receive the weight arena over RCCL (xGMI) -------------
    dtype = {"bf16": wrs.BF16, "f16": wrs.F16, "fp8": wrs.FP8_ENC}[args.dtype]
    t_load = time.time()
    ctx = wrs.WhisperContext(model_path, dtype=dtype, gpu_device=local_rank, load_weights=(rank == 0 or world == 1))
    load_s = time.time() - t_load
    bcast_s = 0.0
    if world > 1:
        uid = C.create_string_buffer(128)
        if rank == 0:
            assert wrs.lib().whisper_mi355x_rccl_unique_id(uid) == 0
        obj = [bytes(uid.raw)]
        dist.broadcast_object_list(obj, src=0)
        barrier()
        t = time.time()
        rc = wrs.lib().whisper_mi355x_broadcast_weights(ctx.ptr, obj[0], rank, world)
        assert rc == 0, rc
        bcast_s = max_over_ranks(time.time() - t, dist, "cuda")
    st = ctx.create_state()

    # ---- this rank's chunks, resident in HBM --------------------------------------------------------
    from make_model import synthetic_pcm
    L = wrs.lib()
    n = 16000 * 30
    if args.batch > 0:
        ids = [rank * args.batch + i for i in range(args.batch)]
        global_batch = args.batch * world
    else:
        ids = rank_chunk_ids(rank, world, args.global_batch)
        global_batch = args.global_batch
    nb = len(ids)
    buf = L.whisper_mi355x_dev_alloc(ctx.ptr, max(1, nb) * n * 4)
    assert buf
    host = np.empty(n, np.float32)
    for i, cid in enumerate(ids):
        host[:] = synthetic_pcm(cid)
        L.whisper_mi355x_memcpy(ctx.ptr, C.c_void_p(buf + i * n * 4), host.ctypes.data, n * 4, 1)
    jobs = [(buf + i * n * 4, n) for i in range(nb)]

    def step(params, fixed=None):
        if nb:
            rc = st.full_batch(params, jobs, on_device=True, fixed_tokens=args.tokens if fixed is None else fixed)
            assert rc == 0, rc

    def timed(params, steps, fixed=None):
        barrier()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(steps):
            step(params, fixed)
        torch.cuda.synchronize()
        barrier()
        return max_over_ranks(time.time() - t0, dist, "cuda")

    params = wrs.reference_full_params("en")
    # warmup (untimed) with every kernel class timed once to find the dominant kernel
    L.whisper_mi355x_kernel_timing(st.ptr, 0xFF)
    tw = time.time()
    for _ in range(args.warmup):
        step(params)
    warm_s = (time.time() - tw) / max(1, args.warmup)
    stats = []
    for k in range(len(K_NAMES)):
        out = (C.c_double * 3)()
        L.whisper_mi355x_kernel_stats(st.ptr, k, out)
        stats.append(tuple(out))
    # the roofline kernel: the largest single kernel. The two GEMM classes hold many kernels (every
    # projection shape and epilogue), so they are excluded; timing one of them would also put an
    # event pair around ~8 launches per layer inside the decode graphs and slow the timed region.
    # Their phases are reported below (roofline.phases) from the phase clocks.
    dom = max(SINGLE_KERNEL, key=lambda k: stats[k][0])
    share = {K_NAMES[k]: round(stats[k][0] / max(1e-9, sum(s[0] for s in stats)), 4) for k in range(len(K_NAMES))}

    # timed region: only the dominant class is event-timed (keeps event overhead off the others)
    # BENCH_KTIME=0: no event pair inside the timed steps (A/B of the instrumentation's own cost)
    # per-layer decode attention classes are sampled every KT_LAYER_STRIDE-th layer: an event pair per
    # launch in all 32 layers cost ~2 % of the step at 128 clips and ~5 % at 16 (BENCH_KTIME=0 A/B)
    mask = (1 << dom) | ((KT_LAYER_STRIDE << 16) if dom in (2, 3) else 0)
    L.whisper_mi355x_kernel_timing(st.ptr, 0 if os.environ.get("BENCH_KTIME") == "0" else mask)
    elapsed = timed(params, args.steps)
    out = (C.c_double * 3)()
    L.whisper_mi355x_kernel_stats(st.ptr, dom, out)
    k_ms, k_cnt, k_work = out[0], out[1], out[2]
    phases = st.phase_ms()
    decoded = L.whisper_mi355x_batch_decoded_tokens(st.ptr)
    L.whisper_mi355x_kernel_timing(st.ptr, 0)

    # the reference's own workloads: the app always passes its default vocabulary as
    # the initial prompt (config.rs:40-42, whisper.rs:98-109) with language "auto" (config.rs:49)
    variants = []
    if args.variants:
        for name, p in (("prompted (default vocabulary, config.rs:40-42), language en",
                         wrs.reference_full_params("en", initial_prompt=wrs.DEFAULT_VOCABULARY)),
                        ("auto language (config.rs:49), no prompt", wrs.reference_full_params(None)),
                        ("reference default: auto language + default vocabulary prompt",
                         wrs.reference_full_params(None, initial_prompt=wrs.DEFAULT_VOCABULARY))):
            step(p)  # warmup (builds the graphs / cross caches of this shape)
            el = timed(p, args.variant_steps)
            variants.append(dict(workload=name, value=round(30.0 * global_batch * args.variant_steps / el, 2),
                                 ms_per_step=round(1e3 * el / args.variant_steps, 2),
                                 prompt_tokens=len(ctx.tokenize(wrs.DEFAULT_VOCABULARY)) if "vocabulary" in name else 0,
                                 phase_ms_last_step={k: round(v, 1) for k, v in st.phase_ms().items()}))
        # SURVEY.md §8d's second mode: real greedy termination (EOT and timestamps end each window),
        # same chunks, same weights. temperature_inc = 0: the greedy attempt's result stands whatever
        # its entropy / logprob (synthetic weights are not trained, so the reference's fallback would
        # re-decode most windows with sampling: --fallback-line 1 adds that verbatim-params line)
        lines = [("real greedy termination (EOT / timestamps end each window; greedy attempt only; "
                  "language en, no prompt)", 0.0)]
        if args.fallback_line:
            lines.append(("whisper.rs:88-124 verbatim (greedy + temperature fallback; language en, no prompt)", 0.2))
        for name, t_inc in lines:
            p = wrs.reference_full_params("en")
            p.temperature_inc = t_inc
            step(p, 0)
            el = timed(p, args.variant_steps, 0)
            dec_tok = L.whisper_mi355x_batch_decoded_tokens(st.ptr)
            fell_back = sum(1 for j in range(nb) for d in st.decisions(j) if d["temp_idx"] > 0)
            variants.append(dict(workload=name, value=round(30.0 * global_batch * args.variant_steps / el, 2),
                                 ms_per_step=round(1e3 * el / args.variant_steps, 2),
                                 decoded_tokens_per_chunk=round(dec_tok / max(1, nb), 1),
                                 windows=sum(len(st.decisions(j)) for j in range(nb)), windows_fallen_back=fell_back,
                                 phase_ms_last_step={k: round(v, 1) for k, v in st.phase_ms().items()}))

        # serving mode: two batches of the same chunks in flight at once, on two whisper_states (each
        # with its own HIP streams and decode graphs) driven from two host threads (ctypes releases the
        # GIL): one batch's launch chain runs in the other's latency gaps. Not the headline (that is one
        # 128-chunk batch at a time, BASELINE configs[3]); tools/overlap_probe.py has the offsets.
        if args.inflight_line and nb:
            import threading
            st2 = ctx.create_state()
            rc2 = [0]

            def step2():
                rc2[0] = st2.full_batch(params, jobs, on_device=True, fixed_tokens=args.tokens)
            step2()
            step(params)
            barrier()
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(args.variant_steps):
                th = threading.Thread(target=step2)
                th.start()
                step(params)
                th.join()
                assert rc2[0] == 0, rc2[0]
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.time() - t0, dist, "cuda")
            variants.append(dict(workload=f"serving: 2 batches of {global_batch} chunks in flight (two states on two "
                                          f"streams, two host threads), fixed {args.tokens}-token decode, language en",
                                 value=round(2 * 30.0 * global_batch * args.variant_steps / el, 2),
                                 ms_per_batch=round(1e3 * el / (2 * args.variant_steps), 2), batches_in_flight=2))
            st2.close()

        # SURVEY.md §8d's clock from PCM on the host: the same step with the chunks handed over as host
        # arrays (whisper_full's own boundary), so the 1.92 MB H2D copy per chunk is inside the timed
        # region. Reported beside `value` (the contract's number has the inputs resident in HBM).
        if nb:
            host_pcm = [synthetic_pcm(cid) for cid in ids]

            def step_host():
                rc = st.full_batch(params, host_pcm, on_device=False, fixed_tokens=args.tokens)
                assert rc == 0, rc
            step_host()
            barrier()
            torch.cuda.synchronize()
            t0 = time.time()
            for _ in range(args.variant_steps):
                step_host()
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.time() - t0, dist, "cuda")
            variants.append(dict(workload="PCM on the host (PCIe-inclusive: H2D copy of every chunk inside the step), "
                                          "language en, no prompt",
                                 value=round(30.0 * global_batch * args.variant_steps / el, 2),
                                 ms_per_step=round(1e3 * el / args.variant_steps, 2), pcie_inclusive=True))
            del host_pcm

    # the f16 engine on the same config: whisper.cpp's own weight type, the parity path (exact against the oracle up to its near ties)
    # (tests/test_gpu_fulldepth.py); bf16 is the headline dtype BASELINE names. One GPU only.
    if args.f16_line and args.dtype == "bf16" and nb and world == 1:
        ctx16 = wrs.WhisperContext(model_path, dtype=wrs.F16, gpu_device=local_rank)
        st16 = ctx16.create_state()

        def step16():
            rc = st16.full_batch(params, jobs, on_device=True, fixed_tokens=args.tokens)
            assert rc == 0, rc
        step16()
        barrier()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(args.variant_steps):
            step16()
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.time() - t0, dist, "cuda")
        variants.append(dict(workload="f16 weights (the GGML file's own type; exact against the oracle up to its near ties), "
                                      "same chunks and fixed-work decode, language en, no prompt", dtype="f16",
                             value=round(30.0 * global_batch * args.variant_steps / el, 2),
                             ms_per_step=round(1e3 * el / args.variant_steps, 2),
                             phase_ms_last_step={k: round(v, 1) for k, v in st16.phase_ms().items()}))
        st16.close()
        ctx16.close()

    frontend = None
    if args.frontend and rank == 0 and nb:
        frontend = bench_frontend(wrs, ctx, buf, nb, n)
    form = st.info()  # the cross-attention form of the timed steps' last call (PMC lookup below)

    if rank == 0:
        audio_s = 30.0 * global_batch * args.steps
        value = audio_s / elapsed
        if k_ms <= 0:  # BENCH_KTIME=0 (instrumentation A/B): no live kernel time
            k_ms, k_cnt = float("nan"), 1
        if K_BOUND[dom] == "mfma":
            achieved = k_work / (k_ms * 1e-3) / 1e12
            roof = dict(bound="mfma", achieved=round(achieved, 2), peak=MFMA_PEAK_TFS, unit="TFLOP/s",
                        frac=round(achieved / MFMA_PEAK_TFS, 4), traffic=None)
        else:
            achieved = k_work / (k_ms * 1e-3) / 1e9
            roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(achieved / HBM_PEAK_GBS, 4), traffic=None)
        grid = None
        if K_NAMES[dom] == "attn_cross_decode":
            from make_model import SHAPES
            grid = cross_step_grid(bool(form["direct"]), nb, SHAPES[args.model][3])
        sym_re = ""
        if K_NAMES[dom] == "pdec_step":
            from make_model import SHAPES
            grid = 256 * 256  # one 256-thread workgroup per CU, whatever the clip count
            # pdec_kernel<T, D, ...>: mangled T is DF16_ (f16) or DF16b (bf16), then Li<D>E
            sym_re = r"pdec_kernelI%s_?Li%dE" % ("DF16" if args.dtype == "f16" else "DF16b", SHAPES[args.model][2])
        traffic, src = pmc_traffic(K_NAMES[dom], form["direct"], grid, sym_re)
        if traffic is not None:
            roof.update(traffic=round(traffic / 1e6, 3), traffic_unit="MB per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)",
                        traffic_source=f"profiles/{src}")
        roof.update(kernel=K_NAMES[dom], launches=int(k_cnt), avg_launch_ms=round(k_ms / max(1, k_cnt), 4),
                    work_per_launch=k_work / max(1, k_cnt), time_share_warmup=share)
        # the decode projection chain (class gemm_decode: the split-K GEMMs with their reduce kernels, the Q'
        # projection, the split merge + Wv, the logits GEMM; the warm-up's 3-token prefill GEMMs too) against HBM:
        # algorithmic bytes (weights + activations + outputs, not the split-K slabs) over its event-timed time in
        # the warm-up step, where every class is timed (VERDICT r5 "next" 2: reported beside the roofline kernel)
        gd_ms, gd_n, gd_w = stats[4]
        if gd_ms > 0:
            gd = gd_w / (gd_ms * 1e-3) / 1e9
            roof["gemm_decode"] = dict(bound="hbm", achieved=round(gd, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                                       frac=round(gd / HBM_PEAK_GBS, 4), calls=int(gd_n),
                                       avg_call_ms=round(gd_ms / max(1, gd_n), 4), source="warm-up step, every class event-timed (a call: a GEMM with its reduce kernel, or one Q-projection / split-merge launch)")
        # per-phase, time-weighted rooflines of rank 0's last step (phase clocks are host wall time
        # around stream-synchronised phases)
        pw = phase_work(args.model, nb, args.tokens, 3, form["direct"])
        enc_s = phases["encode"] * 1e-3
        dec_s = phases["decode"] * 1e-3
        # the encoder's peak: bf16 MFMA; in fp8 mode QKV / FC1 / FC2 run on the fp8 pipe (2x the bf16 rate), so the
        # phase is priced against the time both pipes would need at their peaks (the line had
        # reported the fp8 phase against the bf16 peak alone)
        f8 = pw["enc_flops_fp8"] if args.dtype == "fp8" else 0.0
        ideal_s = (pw["enc_flops"] - f8) / (MFMA_PEAK_TFS * 1e12) + f8 / (FP8_PEAK_TFS * 1e12)
        enc_peak = pw["enc_flops"] / ideal_s / 1e12
        roof["phases"] = {
            "encode": dict(bound="mfma", ms=round(phases["encode"], 1), tflop=round(pw["enc_flops"] / 1e12, 2),
                           achieved=round(pw["enc_flops"] / max(1e-9, enc_s) / 1e12, 1), unit="TFLOP/s",
                           peak=round(enc_peak, 1), frac=round(ideal_s / max(1e-9, enc_s), 4),
                           note=("fp8 mode: %.2f of the %.2f TFLOP on the fp8 pipe (peak %.0f), the rest on bf16 (peak %.0f); "
                                 "peak = the mix's effective peak" % (f8 / 1e12, pw["enc_flops"] / 1e12, FP8_PEAK_TFS, MFMA_PEAK_TFS))
                           if args.dtype == "fp8" else None),
            "decode": dict(bound="hbm", ms=round(phases["decode"], 1), steps=args.tokens - 1,
                           gb_per_step=round(pw["dec_bytes_per_step"] / 1e9, 3),
                           achieved=round(pw["dec_bytes_per_step"] * (args.tokens - 1) / max(1e-9, dec_s) / 1e9, 1),
                           unit="GB/s", peak=HBM_PEAK_GBS,
                           frac=round(pw["dec_bytes_per_step"] * (args.tokens - 1) / max(1e-9, dec_s) / 1e9 / HBM_PEAK_GBS, 4),
                           bytes_split_gb={k: round(pw[k] / 1e9, 3) for k in ("dec_weight_bytes", "dec_cross_bytes", "dec_self_bytes")}),
        }
        if args.quant != "none":  # phase_work prices the decoder weights at 2 B each
            roof["phases"]["decode"]["note"] = f"{args.quant} file: bytes priced as 16-bit weights (the blocks stream fewer)"
        pa, pn = C.c_void_p(), C.c_size_t()
        arena_bytes = pn.value if wrs.lib().whisper_mi355x_weight_arena(ctx.ptr, C.byref(pa), C.byref(pn)) == 0 else None
        app = None
        if args.app_pattern:
            app = []
            try:
                app.append(app_pattern(wrs, args.model_dir, "base+conf", "f16", args.app_calls))
                # f16: the engine's default compute type (capi.cpp whisper_init_*: the GGML file's own type)
                app.append(app_pattern(wrs, args.model_dir, shape, "f16", args.app_calls))
            except Exception as e:  # reported, never fatal to the GPU number
                app.append(dict(error=str(e)))
        cpu = None
        if args.cpu_baseline:
            threads = args.cpu_threads or host_cpu()["usable"]
            try:
                cpu = cpu_baseline(model_path, threads, args.tokens)
            except Exception as e:  # reported, never fatal to the GPU number
                cpu = dict(value=None, unit="audio-sec/s", cores=threads, kind="port", sample=f"failed: {e}")
        scaling = "weak" if args.batch > 0 else "strong"
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "audio-sec/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 2), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": args.dtype,
            "data": ("synthetic (seeded AM-harmonic 30 s PCM; seeded random weights of the named architecture"
                     + (", decoder init as peaked as a trained model's: tools/make_model.py +conf)" if args.weights == "conf"
                        else ")")),
            "config": {"workload": f"{args.model}{'' if args.quant == 'none' else '-' + args.quant} {args.dtype} greedy, "
                                   f"{global_batch} x 30 s chunks per step over "
                                   f"{world} GPU(s) ({nb} on rank 0), fixed {args.tokens}-token decode per chunk, "
                                   f"language en, no prompt",
                       "model": args.model, "quant": None if args.quant == "none" else args.quant,
                       "global_batch": global_batch, "batch_per_gpu": nb,
                       "tokens_per_chunk": args.tokens, "seq_len": 1500,
                       "parallelism": f"dp{world} (chunk sharding, RCCL weight broadcast only)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "variants": variants,
            "app_pattern": app,
            "extra": {"rtf_inverse_per_gpu": round(value / world, 2), "decoded_tokens_per_step": decoded,
                      "cross_form": "direct" if form["direct"] else "cache",
                      "phase_ms_last_step": {k: round(v, 1) for k, v in phases.items()},
                      "warmup_step_s": round(warm_s, 3), "model_load_s": round(load_s, 2),
                      "weight_broadcast_s": round(bcast_s, 3), "frontend": frontend,
                      "pdec_give_ups": L.whisper_mi355x_pdec_give_ups(None),
                      "weight_arena_bytes": arena_bytes},
        }
        print(json.dumps(line), flush=True)
    L.whisper_mi355x_dev_free(ctx.ptr, C.c_void_p(buf))
    st.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
