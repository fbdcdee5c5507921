"""The device range-check build (SURVEY.md §5 race / bounds row): libfdlp_checks.so, compiled with
-DFDLP_DEVICE_CHECKS=1 by __graft_entry__.build(), counts violated range assertions of the index-heavy
kernels -- frame descriptors and reflected sample indices (dct_frame_kernel), the skirt / flat sweep rings
and output rows (ac_vsweep_kernel), straddle windows and partial-chain rows (ac_band_kernel), the LDS image
of durbin4_kernel, the LDS-DMA a rows of the lattice kernel, the OLA slices (ola_log_tiled_kernel) -- in
a device counter.  One child process (the library is chosen when it is loaded) runs the reference golden
sets through every autocorrelation and Durbin path plus the full 1024 x 4 s bench batch; it must stay
silent.  The default library reports the checks as disabled."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECKS_LIB = os.path.join(ROOT, "speech_recognition_tools_amd", "lib", "libfdlp_checks.so")

CHILD = r"""
import json, sys
sys.path.insert(0, %(root)r)
sys.path.insert(0, %(tests)r)
import torch
from conftest import load_golden
from test_gpu_parity import run_gpu
from speech_recognition_tools_amd.plan import device_checks
assert device_checks(reset=True)[0], "not a checks build"
runs = 0
for name in ("wsj", "reverb", "chime4_noise", "mel80", "wsj_diff", "gamma_lifter_odd", "reverb_rir_noise"):
    meta, sig, ref, z = load_golden(name)
    mel = meta["opts"].get("fbank_type", "").startswith("mel")
    for path, lpc in (("auto", "auto"), ("structured_mfma", "lattice8"), ("direct", "lds")):
        if mel and path == "structured_mfma":
            continue  # the structured paths need the cochlear filterbank
        run_gpu(meta, sig, z, path=path, lpc=lpc)
        runs += 1
import bench
from test_bench_shape import _run_batch
_run_batch(bench.scp_list("wsj", 1, 1024, 4.0, 4096, None))
runs += 1
en, v, line = device_checks()
print(json.dumps({"enabled": en, "violations": v, "last_line": line, "runs": runs}))
"""


@pytest.mark.gpu
def test_device_range_checks_silent():
    assert os.path.exists(CHECKS_LIB), "build() compiles libfdlp_checks.so"
    env = dict(os.environ, FDLP_LIB=CHECKS_LIB)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "tests": os.path.join(ROOT, "tests")}],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["enabled"] and res["runs"] == 21
    assert res["violations"] == 0, res


@pytest.mark.gpu
def test_default_library_has_checks_disabled():
    from speech_recognition_tools_amd.plan import device_checks
    assert device_checks() == (False, 0, 0)
