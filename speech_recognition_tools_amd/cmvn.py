"""CMVN statistics on the MI355X: drop-in for Kaldi's `compute-cmvn-stats`, the step right after FDLP
feature extraction in the reference recipes (e2e/wsj/run_fdlp_e1.sh:280, reverb :224, chime4 :193:
`compute-cmvn-stats scp:data/<train>/feats.scp data/<train>/cmvn.ark`).

Kaldi semantics restated (src/featbin/compute-cmvn-stats.cc, src/transform/cmvn.cc AccCmvnStats):
  * stats is a [2, D+1] double matrix; for every frame x (float32):
      stats[0, :D] += x,  stats[1, :D] += x*x (a float32 product),  stats[0, D] += 1.
  * without --spk2utt: one matrix over every utterance of the rspecifier, written as a Kaldi object
    (binary "\\0B" + "DM " by default, text with --binary=false); exit status 1 if no utterance was used;
    utterances whose dimension differs from the first one are counted as errors and skipped.
  * with --spk2utt: one matrix per speaker (spk2utt order), written to a table wspecifier
    (ark:<file> or ark,scp:<ark>,<scp>); utterances missing from the features are warned about.
The accumulation runs on the device (fdlp_cmvn_accumulate, a deterministic two-pass reduction); the
feature arks are read by the native Kaldi matrix reader (fdlp_mat_reader_*) into pinned host buffers
that are double-buffered against the device work.
"""
import argparse
import ctypes
import os
import struct
import sys

import numpy as np
import torch

from ._lib import P_dbl, check, lib


class CmvnAccumulator:
    """Device-resident [2, dim+1] fp64 CMVN stats (Kaldi layout); add() accumulates float32 feature rows."""

    def __init__(self, dim: int, device: int = 0, nspk: int = 0):
        self.dim = int(dim)
        self.dev = torch.device("cuda", device)
        shape = (nspk, 2, self.dim + 1) if nspk else (2, self.dim + 1)
        self.stats = torch.zeros(shape, dtype=torch.float64, device=self.dev)

    def add(self, feats: torch.Tensor, spk: int = None, stream=None):
        if feats.dtype != torch.float32 or not feats.is_cuda or feats.dim() != 2 or feats.shape[1] != self.dim:
            raise ValueError("CmvnAccumulator.add: need a float32 [rows, %d] device tensor" % self.dim)
        feats = feats.contiguous()
        dst = self.stats if spk is None else self.stats[spk]
        s = stream if stream is not None else torch.cuda.current_stream(self.dev)
        check(lib.fdlp_cmvn_accumulate(ctypes.c_void_p(feats.data_ptr()), feats.shape[0], self.dim,
                                       ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(s.cuda_stream)))

    def numpy(self) -> np.ndarray:
        return self.stats.cpu().numpy()


def write_kaldi_dmatrix(path: str, m, binary: bool = True):
    """WriteKaldiObject(Matrix<double>) -- the file compute-cmvn-stats writes for global stats."""
    m = np.ascontiguousarray(m, dtype=np.float64)
    check(lib.fdlp_kaldi_write_dmatrix(path.encode(), m.ctypes.data_as(P_dbl), m.shape[0], m.shape[1],
                                       1 if binary else 0))


def _dmatrix_bytes(m: np.ndarray) -> bytes:
    m = np.ascontiguousarray(m, dtype="<f8")
    return b"\0BDM \x04" + struct.pack("<i", m.shape[0]) + b"\x04" + struct.pack("<i", m.shape[1]) + m.tobytes()


def read_kaldi_dmatrix(path: str) -> np.ndarray:
    """Read a Kaldi double-matrix object (binary DM, or the text form write_kaldi_dmatrix writes)."""
    raw = open(path, "rb").read()
    if raw[:2] == b"\0B":
        if raw[2:5] != b"DM ":
            raise ValueError("%s: not a double matrix" % path)
        r, c = struct.unpack("<i", raw[6:10])[0], struct.unpack("<i", raw[11:15])[0]
        return np.frombuffer(raw[15:15 + 8 * r * c], dtype="<f8").reshape(r, c).copy()
    txt = raw.decode().strip()
    if not (txt.startswith("[") and txt.endswith("]")):
        raise ValueError("%s: not a Kaldi matrix" % path)
    rows = [l.split() for l in txt[1:-1].split("\n") if l.strip()]
    return np.array([[float(v) for v in r] for r in rows], dtype=np.float64).reshape(len(rows), -1)


class MatReader:
    """Iterator over (key, float32 [rows, cols] ndarray) of a Kaldi rspecifier ("scp:..." or "ark:...")."""

    def __init__(self, rspecifier: str):
        self._h = ctypes.c_void_p()
        check(lib.fdlp_mat_reader_open(rspecifier.encode(), ctypes.byref(self._h)))

    def __iter__(self):
        key = ctypes.c_char_p()
        rows, cols = ctypes.c_int32(), ctypes.c_int32()
        data = ctypes.POINTER(ctypes.c_float)()
        while True:
            rc = lib.fdlp_mat_reader_next(self._h, ctypes.byref(key), ctypes.byref(rows), ctypes.byref(cols),
                                          ctypes.byref(data))
            if rc == 0:
                return
            check(rc if rc < 0 else 0)
            n = rows.value * cols.value
            arr = np.ctypeslib.as_array(data, shape=(max(n, 1),))[:n] if n else np.zeros(0, np.float32)
            yield key.value.decode(), arr.reshape(rows.value, cols.value)

    def close(self):
        if self._h:
            lib.fdlp_mat_reader_close(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        self.close()


class _Staging:
    """Two pinned host buffers, each copied to its own device buffer on one stream; the host refills a
    buffer only after the device work that read it has finished (event)."""

    def __init__(self, dim, rows, dev):
        self.rows, self.dim = rows, dim
        self.host = [torch.empty((rows, dim), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        self.devb = [torch.empty((rows, dim), dtype=torch.float32, device=dev) for _ in range(2)]
        self.ev = [None, None]
        self.cur, self.fill = 0, 0

    def room(self):
        return self.rows - self.fill

    def put(self, m):
        if self.fill == 0 and self.ev[self.cur] is not None:
            self.ev[self.cur].synchronize()
        n = m.shape[0]
        self.host[self.cur][self.fill:self.fill + n].numpy()[...] = m
        self.fill += n

    def flush(self, consume):
        if self.fill == 0:
            return
        i, n = self.cur, self.fill
        d = self.devb[i][:n]
        d.copy_(self.host[i][:n], non_blocking=True)
        consume(d)
        self.ev[i] = torch.cuda.Event()
        self.ev[i].record()
        self.cur, self.fill = 1 - i, 0


def compute_global_stats(rspecifier: str, device: int = 0, batch_rows: int = 1 << 19, log=None):
    """(stats [2, D+1] ndarray or None, num_done, num_err) over every utterance of rspecifier."""
    acc, stage = None, None
    num_done = num_err = 0
    for utt, m in MatReader(rspecifier):
        if acc is None:
            torch.cuda.set_device(device)
            acc = CmvnAccumulator(m.shape[1], device)
            stage = _Staging(m.shape[1], batch_rows, acc.dev)
        if m.shape[1] != acc.dim:
            if log:
                log("Dimension mismatch for utterance %s: %d vs. %d" % (utt, m.shape[1], acc.dim))
            num_err += 1
            continue
        pos = 0
        while pos < m.shape[0]:
            take = min(stage.room(), m.shape[0] - pos)
            stage.put(m[pos:pos + take])
            pos += take
            if stage.room() == 0:
                stage.flush(acc.add)
        num_done += 1
    if acc is None:
        return None, num_done, num_err
    stage.flush(acc.add)
    return acc.numpy(), num_done, num_err


def read_spk2utt(rspecifier: str):
    path = rspecifier.split(":", 1)[1] if ":" in rspecifier else rspecifier
    out = []
    for line in open(path):
        t = line.split()
        if t:
            out.append((t[0], t[1:]))
    return out


def compute_spk_stats(rspecifier: str, spk2utt, device: int = 0, log=None):
    """{spk: stats} for the speakers of spk2utt (Kaldi's --spk2utt mode)."""
    where = {}
    for i, (_, utts) in enumerate(spk2utt):
        for u in utts:
            where[u] = i
    acc = None
    dims = {}
    seen = set()
    num_done = num_err = 0
    for utt, m in MatReader(rspecifier):
        if utt not in where:
            continue
        seen.add(utt)
        if acc is None:
            torch.cuda.set_device(device)
            acc = CmvnAccumulator(m.shape[1], device, nspk=len(spk2utt))
        spk = where[utt]
        dims.setdefault(spk, m.shape[1])
        if m.shape[1] != acc.dim:
            num_err += 1
            continue
        acc.add(torch.from_numpy(m).to(acc.dev, non_blocking=False), spk=spk)
        num_done += 1
    for spk, utts in spk2utt:
        for u in utts:
            if u not in seen:
                num_err += 1
                if log:
                    log("Did not find features for utterance %s" % u)
    res = {}
    if acc is not None:
        allst = acc.numpy()
        for i, (spk, _) in enumerate(spk2utt):
            if i in dims:
                res[spk] = allst[i]
            elif log:
                log("No stats accumulated for speaker %s" % spk)
    return res, num_done, num_err


def write_table(wspecifier: str, items):
    """Write {key: double matrix} to "ark:<file>" or "ark,scp:<ark>,<scp>" (binary)."""
    kind, _, rest = wspecifier.partition(":")
    opts = kind.split(",")
    if "ark" not in opts:
        raise ValueError("unsupported wspecifier %s" % wspecifier)
    if "scp" in opts:
        ark_path, scp_path = rest.split(",", 1)
    else:
        ark_path, scp_path = rest, None
    scp_lines = []
    with open(ark_path, "wb") as f:
        for k, m in items:
            f.write(k.encode() + b" ")
            off = f.tell()
            f.write(_dmatrix_bytes(m))
            scp_lines.append("%s %s:%d\n" % (k, os.path.abspath(ark_path), off))
    if scp_path:
        with open(scp_path, "w") as f:
            f.writelines(scp_lines)


def sum_stats_files(paths, out, binary=True):
    """Sum per-JOB global stats objects (the fused --cmvn_stats outputs) into one cmvn.ark."""
    tot = None
    for p in paths:
        m = read_kaldi_dmatrix(p)
        tot = m if tot is None else tot + m
    if tot is None:
        raise ValueError("no stats files")
    write_kaldi_dmatrix(out, tot, binary)
    return tot


def _bool(v):
    if v.lower() in ("true", "1", "yes"):
        return True
    if v.lower() in ("false", "0", "no"):
        return False
    raise argparse.ArgumentTypeError("expected true/false, got %s" % v)


def main(argv=None):
    ap = argparse.ArgumentParser(
        prog="compute-cmvn-stats",
        description="Compute cepstral mean and variance normalization statistics (on the MI355X). "
                    "Usage: compute-cmvn-stats [options] <feats-rspecifier> (<stats-wspecifier>|<stats-wxfilename>)")
    ap.add_argument("--binary", type=_bool, default=True, help="write in binary mode (default true)")
    ap.add_argument("--spk2utt", default="", help="rspecifier for speaker to utterance-list map")
    ap.add_argument("--device", type=int, default=int(os.environ.get("FDLP_DEVICE", "0")))
    ap.add_argument("feats")
    ap.add_argument("stats")
    a = ap.parse_args(argv)
    log = lambda msg: print("WARNING (compute-cmvn-stats) %s" % msg, file=sys.stderr)
    if a.spk2utt:
        res, done, err = compute_spk_stats(a.feats, read_spk2utt(a.spk2utt), a.device, log)
        write_table(a.stats, list(res.items()))
        print("LOG (compute-cmvn-stats) Done accumulating CMVN stats for %d utterances; %d had errors."
              % (done, err), file=sys.stderr)
        return 0 if done else 1
    stats, done, err = compute_global_stats(a.feats, a.device, log=log)
    if stats is None:
        print("ERROR (compute-cmvn-stats) No stats accumulated (no utterances?)", file=sys.stderr)
        return 1
    write_kaldi_dmatrix(a.stats, stats, a.binary)
    print("LOG (compute-cmvn-stats) Wrote global CMVN stats to %s" % a.stats, file=sys.stderr)
    print("LOG (compute-cmvn-stats) Done accumulating CMVN stats for %d utterances; %d had errors."
          % (done, err), file=sys.stderr)
    return 0 if done else 1


if __name__ == "__main__":
    sys.exit(main())
