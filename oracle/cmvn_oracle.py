"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): CPU restatement of Kaldi's CMVN
statistics accumulation, the step after FDLP feature extraction in the reference recipes
(e2e/wsj/run_fdlp_e1.sh:280 `compute-cmvn-stats scp:feats.scp cmvn.ark`).

Kaldi is a third-party dependency absent from /root/reference (its tools/ symlinks dangle), so this
restates its published algorithm -- src/transform/cmvn.cc AccCmvnStats(VectorBase<BaseFloat> feats,
BaseFloat weight, MatrixBase<double>* stats):
    for i < dim:  mean[i] += weight * feats[i];  var[i] += weight * feats[i] * feats[i];   (BaseFloat math)
    mean[dim] += weight
driven frame by frame in utterance order by src/featbin/compute-cmvn-stats.cc (global mode).
No Kaldi binary or golden vector exists here to pin it against: parity unpinned at the Kaldi boundary;
the restatement is checked against hand-computed cases in tests/test_cmvn.py.
"""
import numpy as np


def acc_cmvn_stats(frames, stats=None):
    """frames: float32 [T, D] (one utterance); stats: [2, D+1] float64 accumulated in place (Kaldi order:
    sequential over frames, float32 squares)."""
    x = np.asarray(frames, dtype=np.float32)
    if stats is None:
        stats = np.zeros((2, x.shape[1] + 1), dtype=np.float64)
    if x.shape[0] == 0:
        return stats
    sq = (x * x).astype(np.float32)  # weight (1.0f) * f * f in BaseFloat
    # np.cumsum is a strictly sequential float64 accumulation, like Kaldi's frame loop
    s = np.cumsum(np.vstack([stats[0, :-1][None, :], x.astype(np.float64)]), axis=0)[-1]
    q = np.cumsum(np.vstack([stats[1, :-1][None, :], sq.astype(np.float64)]), axis=0)[-1]
    stats[0, :-1] = s
    stats[1, :-1] = q
    stats[0, -1] += float(x.shape[0])
    return stats


def global_stats(utterances):
    """compute-cmvn-stats (no --spk2utt) over an iterable of [T, D] float32 matrices in order."""
    stats = None
    for m in utterances:
        stats = acc_cmvn_stats(m, stats)
    return stats
