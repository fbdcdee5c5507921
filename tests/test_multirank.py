"""The N>1 path on CPU (gloo, world_size 2): scp sharding and the bench's timed region.

Utterances shard across ranks with no data-path collective; the only cross-rank
traffic is the barrier and the max-of-elapsed all-reduce of bench.py's timed region.  Each rank here
featurises its shard with the oracle (a CPU stand-in for the GPU plan: this checks the sharding and the
harness, not the kernels), and the gathered per-utterance results must equal a one-process run of each
JOB shard (every JOB owns its jitter RNG stream, like the reference's JOB processes)."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as tmp

from speech_recognition_tools_amd import shard


def test_split_counts_like_split_scp():
    assert shard.split_counts(10, 3) == [4, 3, 3]
    assert shard.split_counts(3, 3) == [1, 1, 1]
    lines = ["u%d p\n" % i for i in range(11)]
    parts = shard.split_lines(lines, 4)
    assert [len(p) for p in parts] == [3, 3, 3, 2]
    assert sum(parts, []) == lines
    assert shard.shard_of(lines, 3, 4) == lines[9:]
    with pytest.raises(ValueError):
        shard.split_counts(2, 3)


def test_split_lists_files(tmp_path):
    src = tmp_path / "wav.scp"
    src.write_text("".join("utt%02d /x/%d.wav\n" % (i, i) for i in range(7)))
    outs = [str(tmp_path / ("wav.%d.scp" % n)) for n in (1, 2, 3)]
    shard.split_lists(str(src), outs)
    got = [open(o).read() for o in outs]
    assert "".join(got) == src.read_text()
    assert [g.count("\n") for g in got] == [3, 2, 2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _utts(n):
    rng = np.random.default_rng(5)
    lens = rng.integers(8000, 30000, n)
    return [("utt%02d" % i, np.clip(np.round(rng.standard_normal(int(T)) * 1500), -32768, 32767).astype(np.int16))
            for i, T in enumerate(lens)]


def _rank_main(rank, world, port, n_utt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from oracle import fdlp_oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard.shard_of(_utts(n_utt), rank, world)
    orc = O.FdlpOracle(O.FdlpConfig.wsj())
    res = {}

    def step():
        rng = random.Random(100 + rank)  # the JOB's own jitter stream, restarted per pass
        for u, x in mine:
            res[u] = orc.utterance(x, rng)

    local = []

    def timed_step():
        import time
        t = time.perf_counter()
        step()
        local.append(time.perf_counter() - t)

    el = shard.timed_steps(timed_step, 2, 1, lambda: None, dist, torch.device("cpu"))
    gathered = [None] * world
    dist.all_gather_object(gathered, {u: float(np.sum(v)) for u, v in res.items()})
    dist.destroy_process_group()
    q.put((rank, el, sum(local[1:]), gathered))


def test_two_rank_gloo_shards_and_timed_region():
    world, n_utt = 2, 5
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n_utt, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out.sort()
    # max over ranks: every rank reports the same elapsed, and it bounds each rank's own step time
    assert out[0][1] == out[1][1]
    for _, el, own, _ in out:
        assert el >= own * 0.999
    # shards are disjoint and cover the scp; results equal a one-process run of each JOB shard
    merged = {}
    for part in out[0][3]:
        assert not set(part) & set(merged)
        merged.update(part)
    utts = _utts(n_utt)
    assert sorted(merged) == [u for u, _ in utts]
    from oracle import fdlp_oracle as O
    orc = O.FdlpOracle(O.FdlpConfig.wsj())
    for r in range(world):
        rng = random.Random(100 + r)
        for u, x in shard.shard_of(utts, r, world):
            assert merged[u] == float(np.sum(orc.utterance(x, rng)))
