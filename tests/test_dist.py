"""Multi-rank path on the CPU (gloo, world_size 2 and 4).

1. bench.py's own launcher: `bench.py --gpus N --plan` spawns N rank processes (the path the
   driver's `--gpus N` takes without torchrun), each joins the process group, takes its
   strong-scaling shard of the global batch (ceil(B/n) contiguous chunks per rank),
   and rank 0 reports the max over ranks of a rank-dependent time.
2. Transcribing each rank's shard independently gives exactly the single-process result for every
   chunk (no data-path collective). The per-chunk transcription here is the CPU oracle
   (test infrastructure) standing in for the GPU engine, which these CPU tests cannot run; the
   engine's own multi-rank piece, the RCCL weight broadcast, is covered by tests/test_gpu_dist.py.
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BATCH = 5  # global batch: ranks get ceil(5/2) = 3 and 2 chunks


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_launcher_strong_shards(world):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--plan",
                          "--global-batch", "128"], capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["world"] == world
    assert line["max_elapsed"] == 0.25 * world
    shards = line["shards"]
    per = -(-128 // world)
    assert [len(s) for s in shards] == [per] * world
    assert sorted(c for s in shards for c in s) == list(range(128))
    assert all(s == list(range(r * per, (r + 1) * per)) for r, s in enumerate(shards))


def test_rank_chunk_ids_ragged():
    sys.path.insert(0, ROOT)
    import bench
    assert [bench.rank_chunk_ids(r, 3, 8) for r in range(3)] == [[0, 1, 2], [3, 4, 5], [6, 7]]
    assert [bench.rank_chunk_ids(r, 8, 128) for r in (0, 7)] == [list(range(16)), list(range(112, 128))]
    assert bench.rank_chunk_ids(3, 4, 3) == []


def _transcribe(model, cid):
    from make_model import synthetic_pcm
    from oracle_py import Oracle, reference_params
    o = Oracle(model, mode=1, n_threads=2)
    r = o.full(synthetic_pcm(cid, seconds=5), reference_params("en", fixed_tokens=6))
    o.close()
    assert r["rc"] == 0
    return [(s["t0"], s["t1"], s["text"], list(s["tokens"])) for s in r["segments"]]


def _worker(rank, world, port, model, q):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests"), os.path.join(root, "tools")]
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = bench.rank_chunk_ids(rank, world, BATCH)
    res = {cid: _transcribe(model, cid) for cid in ids}
    gathered = [None] * world
    dist.all_gather_object(gathered, res)
    t = bench.max_over_ranks(float(rank + 1) * 0.5, dist, "cpu")
    if rank == 0:
        q.put((gathered, t))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_single_process(micro_model):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, micro_model, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 1.0  # max over ranks of 0.5, 1.0
    merged = {}
    for part in gathered:
        assert not (set(part) & set(merged)), "ranks transcribed overlapping chunks"
        merged.update(part)
    assert sorted(merged) == list(range(BATCH))
    assert [len(p) for p in gathered] == [3, 2]
    for cid, r in merged.items():
        assert r == _transcribe(micro_model, cid), f"chunk {cid}"
