"""extract-segments: drop-in for the Kaldi tool the reference driver calls when a data directory has a
`segments` file (recipes/timit/local_pyspeech/make_FDLPspectrum_feats.sh:126-129):

    extract-segments [--min-segment-length=0.1] [--max-overshoot=0.5] \\
        scp,p:<wav.scp> <segments> ark,scp:<dump.ark>,<dump.scp>

It cuts every segment `<utt> <recording> <start-sec> <end-sec> [<channel>]` out of its recording and
writes it as a Kaldi wave archive (key, space, a canonical PCM16 RIFF file), which
compute-fdlp-feats --scp_type segment then reads natively (io_pipeline.read_rx: `<ark>:<offset>`).

Kaldi itself is absent here; the rules restated from its published extract-segments.cc
(src/featbin) are: start_samp = trunc(start * fs), end_samp = trunc(end * fs) (end = -1: to the end);
invalid times, a start past the end of the recording, an end more than max_overshoot seconds past it,
or a segment shorter than min_segment_length seconds are skipped with a warning; a small overshoot is
truncated to the recording.  Parity with Kaldi's own output is unpinned (no Kaldi binary or fixture).
"""
import argparse
import os
import struct
import sys

import numpy as np


def riff_bytes(samples: np.ndarray, sr: int) -> bytes:
    """Canonical 44-byte-header PCM16 RIFF (what Kaldi's WaveData::Write produces)."""
    x = np.asarray(samples, dtype="<i2")
    ch = 1 if x.ndim == 1 else x.shape[1]
    data = x.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE" + b"fmt " + struct.pack(
        "<IHHIIHH", 16, 1, ch, sr, sr * ch * 2, ch * 2, 16) + b"data" + struct.pack("<I", len(data))
    return hdr + data


def _table_path(spec: str) -> str:
    return spec.split(":", 1)[1] if ":" in spec else spec


def segment_bounds(start: float, end: float, num_samp: int, fs: float, min_len: float, max_over: float):
    """(start_samp, end_samp) or (None, reason) following extract-segments.cc."""
    if start < 0 or (end != -1 and end <= 0) or (start >= end and end > 0):
        return None, "invalid segment times"
    s = int(start * fs)
    e = int(end * fs) if end != -1 else num_samp
    if s < 0 or s >= num_samp:
        return None, "start sample out of range"
    if e > num_samp:
        if e >= num_samp + int(max_over * fs):
            return None, "end sample too far out of range"
        e = num_samp
    if (e - s) < min_len * fs:
        return None, "segment too short"
    return (s, e), None


def extract_segments(wav_rspec: str, segments: str, wav_wspec: str, min_len: float = 0.1,
                     max_over: float = 0.5, log=None):
    """Returns (num_done, num_skipped)."""
    from .io_pipeline import read_rx_bytes
    from .featgen.features import read_wav_bytes
    recs = {}
    for line in open(_table_path(wav_rspec)):
        t = line.strip().split(None, 1)
        if len(t) == 2:
            recs[t[0]] = t[1]
    kind, _, rest = wav_wspec.partition(":")
    opts = kind.split(",")
    if "ark" not in opts:
        raise ValueError("unsupported wspecifier " + wav_wspec)
    ark_path, scp_path = (rest.split(",", 1) if "scp" in opts else (rest, None))
    cache_key, cache = None, None
    done = skipped = 0
    scp_lines = []
    warn = log or (lambda m: print("WARNING (extract-segments) " + m, file=sys.stderr))
    with open(ark_path, "wb") as ark:
        for line in open(segments):
            t = line.split()
            if not t:
                continue
            if len(t) not in (4, 5):
                warn("Invalid line in segments file: " + line.strip())
                skipped += 1
                continue
            seg, rec = t[0], t[1]
            try:
                start, end = float(t[2]), float(t[3])
            except ValueError:
                warn("Invalid line in segments file: " + line.strip())
                skipped += 1
                continue
            if rec not in recs:
                warn("Could not find recording %s, skipping segment %s" % (rec, seg))
                skipped += 1
                continue
            if rec != cache_key:
                try:
                    cache = read_wav_bytes(read_rx_bytes(recs[rec]))
                except Exception:
                    cache = None
                cache_key = rec
            if cache is None:
                warn("Could not read recording %s, skipping segment %s" % (rec, seg))
                skipped += 1
                continue
            sr, x = cache
            if x.ndim == 1:
                x = x[:, None]
            if len(t) == 5:
                c = int(t[4])
                if c >= x.shape[1]:
                    warn("Invalid channel %d >= %d for segment %s" % (c, x.shape[1], seg))
                    skipped += 1
                    continue
                x = x[:, c:c + 1]
            b, why = segment_bounds(start, end, x.shape[0], float(sr), min_len, max_over)
            if b is None:
                warn("%s for segment %s" % (why, seg))
                skipped += 1
                continue
            piece = x[b[0]:b[1]]
            ark.write(seg.encode() + b" ")
            off = ark.tell()
            ark.write(riff_bytes(piece[:, 0] if piece.shape[1] == 1 else piece, sr))
            scp_lines.append("%s %s:%d\n" % (seg, os.path.abspath(ark_path), off))
            done += 1
    if scp_path:
        with open(scp_path, "w") as f:
            f.writelines(scp_lines)
    return done, skipped


def main(argv=None):
    ap = argparse.ArgumentParser(prog="extract-segments",
                                 description="Extract segments from a wav archive (Kaldi extract-segments drop-in)")
    ap.add_argument("--min-segment-length", "--min_segment_length", type=float, default=0.1)
    ap.add_argument("--max-overshoot", "--max_overshoot", type=float, default=0.5)
    ap.add_argument("wav_rspecifier")
    ap.add_argument("segments")
    ap.add_argument("wav_wspecifier")
    a = ap.parse_args(argv)
    done, skipped = extract_segments(a.wav_rspecifier, a.segments, a.wav_wspecifier, a.min_segment_length,
                                     a.max_overshoot)
    print("LOG (extract-segments) Successfully processed %d lines out of %d in the segments file."
          % (done, done + skipped), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
