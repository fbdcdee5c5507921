"""Host input/output runtime of the FDLP path: the part of getFeats that is not
DSP -- reading utterances (computeFDLPSpectrogram.py:119-154) and writing the ark (:231) -- arranged so
the host keeps the MI355X busy:

  * PrefetchReader: a bounded thread pool reads and parses the scp entries ahead of the consumer, in
    scp order.  Entries are `<path>`, `<cmd> |` (pipes, e.g. sph2pipe), and Kaldi wave-archive
    rxspecifiers `<ark>:<offset>` (what extract-segments writes and `--scp_type segment` lists); the
    RIFF parse is native (fdlp_wav_parse, the GIL is released during ctypes calls and file reads).
  * read_rx: one entry; `--scp_type segment` entries are read natively too (the reference shells out to
    Kaldi `wav-copy <rx> -`, which must be on PATH there).
  * ArkStream: the native Kaldi ark/scp writer, fed utterance by utterance as batches complete, so a
    JOB never holds all of its features in memory (the reference builds one dict of every utterance).
"""
import collections
import ctypes
import os
import re
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ._lib import check, lib, ptr
from .featgen.features import read_wav_bytes

_ARK_OFFSET = re.compile(r"^(.*):(\d+)$")


def read_rx_bytes(rx: str) -> bytes:
    """Bytes of the RIFF file an scp entry designates: '<cmd> |', '<ark>:<offset>' or '<path>'."""
    rx = rx.strip()
    if rx.endswith("|"):
        proc = subprocess.run(rx[:-1], shell=True, stdout=subprocess.PIPE)
        return proc.stdout
    m = _ARK_OFFSET.match(rx)
    if m and os.path.isfile(m.group(1)) and not os.path.isfile(rx):
        with open(m.group(1), "rb") as f:
            f.seek(int(m.group(2)))
            head = f.read(8)
            if head[:4] != b"RIFF":
                raise ValueError("no RIFF wave at %s" % rx)
            size = int.from_bytes(head[4:8], "little")
            return head + f.read(size)
    with open(rx, "rb") as f:
        return f.read()


def read_rx(line: str, scp_type: str):
    """(uttid, int16 samples, sr) of one scp line, or (uttid, None, None) when reading fails (the
    reference skips such utterances, computeFDLPSpectrogram.py:129-154)."""
    tokens = line.strip().split()
    uttid, rx = tokens[0], " ".join(tokens[1:])
    if scp_type not in ("wav", "segment"):
        raise ValueError("Invalid type of scp type, it should be either wav or segment")
    try:
        sr, sig = read_wav_bytes(read_rx_bytes(rx))
        return uttid, sig, sr
    except Exception:
        return uttid, None, None


class PrefetchReader:
    """Iterates (uttid, samples, sr) over the non-empty lines of an scp file in order.

    scps with `<cmd> |` entries (sph2pipe & co., one subprocess each) are read up to `depth` entries
    ahead on `workers` threads.  Plain files and ark offsets are read inline: the per-entry work is a
    ~128 KB read and a native RIFF parse, and a pool of per-entry futures costs more in GIL hand-offs
    than it overlaps (MI355X box, benchmarks/cli_throughput.py, 2048 x 4 s: 8.2 / 6.9 audio-h/s
    inline against 6.1 / 5.6 with 4 pooled threads)."""

    def __init__(self, scp_path: str, scp_type: str = "wav", workers: int = 4, depth: int = 64):
        if scp_type not in ("wav", "segment"):
            raise ValueError("Invalid type of scp type, it should be either wav or segment")
        self.scp_path, self.scp_type = scp_path, scp_type
        self.workers, self.depth = max(1, int(workers)), max(1, int(depth))

    def __iter__(self):
        with open(self.scp_path, "r") as fid:
            lines = [l for l in fid if l.strip()]
        if self.workers == 1 or not any(l.rstrip().endswith("|") for l in lines):
            for l in lines:
                yield read_rx(l, self.scp_type)
            return
        with ThreadPoolExecutor(max_workers=self.workers) as pool:
            q = collections.deque()
            for l in lines:
                q.append(pool.submit(read_rx, l, self.scp_type))
                if len(q) >= self.depth:
                    yield q.popleft().result()
            while q:
                yield q.popleft().result()


class ArkStream:
    """Kaldi binary ark + scp written as utterances complete (native fdlp_ark_* writer)."""

    def __init__(self, outfile: str):
        self._h = ctypes.c_void_p()
        check(lib.fdlp_ark_open((outfile + ".ark").encode(), (outfile + ".scp").encode(), ctypes.byref(self._h)))
        self._lock = threading.Lock()

    def write(self, key: str, feat: np.ndarray):
        m = np.ascontiguousarray(feat, dtype=np.float32)
        if m.ndim != 2:
            raise ValueError("feature matrix must be 2-D")
        with self._lock:
            check(lib.fdlp_ark_write(self._h, key.encode(), ptr(m, ctypes.c_float), m.shape[0], m.shape[1]))

    def close(self):
        """Publish: rename the .tmp files to their final names."""
        if self._h:
            h, self._h = self._h, ctypes.c_void_p()
            check(lib.fdlp_ark_close(h))

    def abort(self):
        """Failure path: delete the .tmp files, publish nothing (fdlp_ark_abort)."""
        if self._h:
            h, self._h = self._h, ctypes.c_void_p()
            lib.fdlp_ark_abort(h)

    def finish(self, ok: bool):
        self.close() if ok else self.abort()

    def __enter__(self):
        return self

    def __exit__(self, exc_type, *exc):
        self.finish(exc_type is None)
