"""PyTorch-ROCm operator over the C ABI ("a thin op wrapping fdlp_compute on tensors"):

    torch.ops.fdlp.spectrogram(plan_id, pcm, lengths, jitter, ark_decimals) -> float32 [sum L, out_dim]

* ``plan_id``  -- FdlpPlan.op_id (plans register themselves; the op looks the plan up by id)
* ``pcm``      -- int16 or float64 device tensor, the utterances' samples concatenated
* ``lengths``  -- int64 host tensor [n_utt] of samples per utterance (getFrames / ceil(T frate / srate))
* ``jitter``   -- uint8 host tensor of the concatenated randrange(2) hop draws, F_u - 1 per utterance
                  (computeFDLPSpectrogram.py:225; PyRandom.randbits2)
* ``ark_decimals`` -- the reference's '%.3f' text-ark rounding (3), -1 keeps full float32

It runs fdlp_compute on the current stream of the pcm's device (the HIP kernels of libfdlp_hip.so; no
fallback).  The output row count depends on the lengths' values, so the fake (meta) kernel declares a
data-dependent size.
"""
import weakref

import numpy as np
import torch

_PLANS = weakref.WeakValueDictionary()
_NEXT = [1]


def register_plan(plan) -> int:
    pid = _NEXT[0]
    _NEXT[0] += 1
    _PLANS[pid] = plan
    return pid


@torch.library.custom_op("fdlp::spectrogram", mutates_args=())
def spectrogram(plan_id: int, pcm: torch.Tensor, lengths: torch.Tensor, jitter: torch.Tensor,
                ark_decimals: int) -> torch.Tensor:
    plan = _PLANS.get(int(plan_id))
    if plan is None:
        raise ValueError("fdlp::spectrogram: unknown plan id %d" % plan_id)
    lens = lengths.detach().cpu().numpy().astype(np.int64)
    jit = jitter.detach().cpu().numpy().astype(np.uint8)
    out, rows, _ = plan.compute(pcm, lens, jit, ark_decimals=int(ark_decimals))
    return out


@spectrogram.register_fake
def _spectrogram_fake(plan_id, pcm, lengths, jitter, ark_decimals):
    plan = _PLANS.get(int(plan_id))
    dim = plan.out_dim if plan is not None else 1
    rows = torch.library.get_ctx().new_dynamic_size()
    return pcm.new_empty((rows, dim), dtype=torch.float32)
