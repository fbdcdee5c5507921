import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfdlp_hip.so on the device)")


def load_golden(name):
    """(meta, signals dict, reference outputs dict, raw npz) of a fixture made by make_golden.py."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    meta = json.loads(str(z["meta"]))
    sig = {u: z["in_" + u] for u in meta["utts"]}
    ref = {u: z["out_" + u] for u in meta["utts"]}
    return meta, sig, ref, z


GOLDEN_SETS = ["wsj", "reverb", "chime4_noise", "cli_default_mel", "mel80", "wsj_diff", "gamma_lifter_odd",
               "reverb_rir", "reverb_rir_noise", "wav_kinds_noise", "wav_kinds_diff"]


def oracle_cfg(meta):
    from oracle import fdlp_oracle as O
    o = meta["opts"]
    cfg = O.FdlpConfig(nfilters=o["nfilters"], coeff_num=o["coeff_num"], coeff_range=o["coeff_range"],
                       order=o["order"], fduration=o["fduration"], frate=o["frate"],
                       overlap_fraction=o["overlap_fraction"], fbank_type=o["fbank_type"],
                       odd_mod_zero=o.get("odd_mod_zero", False), gamma_weight=o.get("gamma_weight", "None"))
    if "lifter" in meta["extra"]:
        cfg.lifter = np.array(meta["extra"]["lifter"])
    return cfg


def feature_cfg(meta, support_eps=None):
    from speech_recognition_tools_amd import FeatureConfig, DEFAULT_SUPPORT_EPS
    o = meta["opts"]
    return FeatureConfig(nfilters=o["nfilters"], coeff_num=o["coeff_num"], coeff_range=o["coeff_range"],
                         order=o["order"], fduration=o["fduration"], frate=o["frate"],
                         overlap_fraction=o["overlap_fraction"], fbank_type=o["fbank_type"],
                         odd_mod_zero=o.get("odd_mod_zero", False), gamma_weight=o.get("gamma_weight", "None"),
                         lifter=meta["extra"].get("lifter"),
                         support_eps=DEFAULT_SUPPORT_EPS if support_eps is None else support_eps)
