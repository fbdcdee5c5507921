"""bench.py's N > 1 path on the CPU: `--gpus N` without a launcher starts N rank processes itself,
every rank takes a contiguous split_scp shard of the synthetic scp (make_FDLPspectrum_feats.sh:135-157),
ranks meet over gloo for the barrier and the max-of-elapsed only, and rank 0 prints one JSON line.
--dry-run skips the device work and keeps the launcher, the sharding and the reduction."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2", "--warmup", "1"]
                       + list(extra), cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_dry_run_shards_cover_scp(gpus):
    res = _run("--gpus", str(gpus), "--utts", "5")
    assert res["n_gpus"] == gpus and res["dry_run"]
    assert res["scp_entries"] == 5 * gpus
    shards = res["shards"]
    assert len(shards) == gpus
    assert shards[0][0] == 0 and shards[-1][1] == res["scp_entries"]
    for (a0, a1, fa), (b0, b1, fb) in zip(shards, shards[1:]):
        assert a1 == b0 and a0 < a1                      # contiguous, disjoint, non-empty
    assert all(f == 5 * 4 for _, _, f in shards)         # 5 utterances x 4 frames of 4 s each


def test_dry_run_librispeech_shards_balance_frames():
    res = _run("--gpus", "2", "--workload", "librispeech", "--frames", "300")
    shards = res["shards"]
    assert shards[0][1] == shards[1][0] and shards[1][1] == res["scp_entries"]
    tot = sum(f for _, _, f in shards)
    assert tot <= 600 and all(f >= 0.3 * tot for _, _, f in shards)


@pytest.mark.parametrize("gpus", [1, 2])
def test_every_rank_gets_its_pcie_child(gpus):
    """The PCIe-inclusive pass (with_transfers, SURVEY 8(d) "first H2D to last D2H") runs in a child process
    of every rank, started before the rank touches the GPU: single-process argv over the rank's own shard,
    GPU_MAX_HW_QUEUES raised, the rank's GPU only, no rendezvous variables."""
    res = _run("--gpus", str(gpus), "--utts", "5")
    ch = res["xfer_children"]
    assert len(ch) == gpus
    for r, c in enumerate(ch):
        a = c["argv"]
        assert "--xfer-only" in a and "--dry-run" not in a
        assert a[a.index("--gpus") + 1] == "1" and a.count("--gpus") == 1
        assert a[a.index("--xfer-shard") + 1] == "%d/%d" % (r, gpus)
        assert c["env"]["GPU_MAX_HW_QUEUES"] == "8"
        assert c["env"]["HIP_VISIBLE_DEVICES"] == (str(r) if gpus > 1 else os.environ.get("HIP_VISIBLE_DEVICES"))
        assert c["rank_env_dropped"] and c["before_gpu_init"]


def test_pcie_children_combine():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    got = [{"value": 10.0, "audio_h": 1.0, "elapsed_s": 0.1, "ms_per_step": 10.0, "note": "n"},
           {"value": 8.0, "audio_h": 1.0, "elapsed_s": 0.125, "ms_per_step": 12.5, "note": "n"}]
    x = b.combine_xfer_children(got)
    assert abs(x["value"] - 16.0) < 1e-12 and x["ms_per_step"] == 12.5 and x["per_rank_value"] == [10.0, 8.0]
    assert b.combine_xfer_children([got[0], None]) is None
    # with the children's absolute start times: the union of their timed regions (a late start lengthens it)
    got[0]["t_go"], got[1]["t_go"] = 100.0, 100.05
    x = b.combine_xfer_children(got)
    assert abs(x["elapsed_s"] - 0.175) < 1e-9 and abs(x["value"] - 2.0 / 0.175) < 1e-9
    assert abs(x["start_spread_s"] - 0.05) < 1e-9 and abs(x["ms_per_step"] - 17.5) < 1e-9 and "t_go" not in x


def test_bench_help_lists_only_live_options():
    """the schedule variants measured at or below the default are gone from bench.py."""
    b = _bench_module()
    a = b.parse_args([])
    for gone in ("xfer_procs", "xfer_sets", "xfer_schedule", "xfer_threads", "xfer_h2d_streams", "xfer_variants",
                 "xfer_compute_streams", "pipeline", "ola_path"):
        assert not hasattr(a, gone), gone
    a, _ = b.xfer_child_spec(a, 1, 0, 0, argv=[], environ={})
    assert a[a.index("--xfer-shard") + 1] == "0/1"


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    return b


@pytest.mark.parametrize("environ,local,want", [
    ({"HIP_VISIBLE_DEVICES": "4,5,6,7"}, 1, "5"),
    ({"CUDA_VISIBLE_DEVICES": "2,3"}, 1, "3"),                              # a pool that sets only CUDA_*
    ({"HIP_VISIBLE_DEVICES": "6,7", "CUDA_VISIBLE_DEVICES": "0,1"}, 0, "6"),  # HIP's list wins, as in HIP
    ({}, 3, "3"),
])
def test_pcie_child_lands_on_the_ranks_gpu(environ, local, want):
    """The child of rank `local` sees exactly the rank's physical GPU through HIP_VISIBLE_DEVICES, whichever
    of HIP_/CUDA_VISIBLE_DEVICES the pool set, and no CUDA_VISIBLE_DEVICES that HIP could re-index."""
    b = _bench_module()
    args = b.parse_args(["--gpus", "4"])
    _, env = b.xfer_child_spec(args, 4, local, local, argv=["--gpus", "4"], environ=environ)
    assert env["HIP_VISIBLE_DEVICES"] == want and "CUDA_VISIBLE_DEVICES" not in env


def test_cpu_workers_default_is_capped(monkeypatch):
    b = _bench_module()
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    n, rule = b.host_cores(with_rule=True)
    assert 1 <= n <= b.CPU_WORKERS_CAP and "unset" in rule
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    n, rule = b.host_cores(with_rule=True)
    assert n == min(3, len(os.sched_getaffinity(0))) and "OMP_NUM_THREADS 3" in rule
