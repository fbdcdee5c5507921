"""Multi-GPU sharding of the FDLP path: utterances are independent, so a job splits its
scp into contiguous balanced shards (like Kaldi's utils/split_scp.pl, which the reference driver
make_FDLPspectrum_feats.sh:126-136 calls) and runs one process per GPU on its shard.  There is no
collective on the data path; the only cross-rank traffic is the bench's barrier and its max-of-elapsed.

No torch / library import at module level: the driver script calls split_lists() from a plain python3.
"""
import glob
import os
import time


def visible_gpu_count():
    """GPUs this process may use, without initialising HIP: the first of HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES that is set (its entry count), else the KFD topology's
    GPU nodes (gpu_id != 0).  The same rule as scripts/make_FDLPspectrum_feats.sh's visible_gpus."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip()])
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(f) as fh:
                n += int(fh.read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    return n


def split_counts(n, k):
    """Sizes of k contiguous shards of n lines: the first n % k shards get one extra line
    (utils/split_scp.pl's balanced split).  Raises like split_scp.pl when n < k."""
    if k <= 0:
        raise ValueError("split_scp: number of shards must be positive")
    if n < k:
        raise ValueError("split_scp: fewer lines (%d) than jobs (%d)" % (n, k))
    return [n // k + (1 if i < n % k else 0) for i in range(k)]


def split_lines(lines, k):
    """lines -> list of k contiguous shards (order preserved, concatenation == lines)."""
    out, pos = [], 0
    for m in split_counts(len(lines), k):
        out.append(lines[pos:pos + m])
        pos += m
    return out


def shard_of(lines, rank, world):
    """The shard rank `rank` of `world` processes owns."""
    return split_lines(lines, world)[rank]


def split_lists(src, outs):
    """split_scp.pl <src> <out1> ... <outk>: write the k shards of file src (lines kept verbatim)."""
    with open(src) as f:
        lines = f.read().splitlines(True)
    for path, part in zip(outs, split_lines(lines, len(outs))):
        with open(path, "w") as f:
            f.writelines(part)


def timed_steps(step, steps, warmup, sync, dist=None, device=None, before_timed=None):
    """The bench contract's timed region: `warmup` untimed steps, then exactly `steps` steps bracketed by
    a barrier and a device sync on both sides; returns the MAX elapsed seconds over ranks.

    step:   callable running one pass of the hot path over this rank's batch
    sync:   callable that waits for this rank's device work (torch.cuda.synchronize, or a no-op on CPU)
    dist:   torch.distributed (initialised) when world > 1, else None
    device: where the max-reduction tensor lives (cuda for nccl/RCCL, cpu for gloo)
    before_timed: optional hook run after the warmup (e.g. switch on per-stage HIP-event timing)
    """
    for _ in range(warmup):
        step()
    sync()
    if before_timed is not None:
        before_timed()
    multi = dist is not None and dist.is_initialized() and dist.get_world_size() > 1
    if multi:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if multi:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


if __name__ == "__main__":
    import sys
    if len(sys.argv) < 3:
        sys.exit("usage: shard.py <scp> <out1> [<out2> ...]")
    try:
        split_lists(sys.argv[1], sys.argv[2:])
    except ValueError as e:
        sys.exit(str(e))
