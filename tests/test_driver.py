"""scripts/make_FDLPspectrum_feats.sh on the CPU: with a Kaldi-style $cmd launcher (--cmd run.pl-like)
every JOB gets --device_rr=JOB,<ngpu> so JOB n runs on GPU (n-1) mod ngpu (the reference's recipes call
the driver with --cmd "$train_cmd", e2e/wsj/run_fdlp_e1.sh:189-209); the CLI resolves it before any GPU
call.  A fake run.pl records the command lines instead of running them."""
import os
import sys
import subprocess

import pytest

from conftest import ROOT


def _resolve(argv):
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import build_parser, resolve_device
    return resolve_device(build_parser().parse_args(argv))


def test_resolve_device_options(monkeypatch):
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    assert _resolve(["a.scp", "o"]) == 0
    assert _resolve(["a.scp", "o", "--device_rr=7,4"]) == 2
    assert _resolve(["a.scp", "o", "--device_rr=7,4", "--device=1"]) == 1
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert _resolve(["a.scp", "o"]) == 3
    with pytest.raises(ValueError):
        _resolve(["a.scp", "o", "--device_rr=0,4"])
    # a scheduler that hands each JOB its own GPU: the round-robin index folds into what the JOB sees
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    assert _resolve(["a.scp", "o", "--device_rr=7,4"]) == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,3")
    assert _resolve(["a.scp", "o", "--device_rr=7,4"]) == 0
    assert _resolve(["a.scp", "o", "--device_rr=4,4"]) == 1


def test_visible_gpu_count(monkeypatch):
    from speech_recognition_tools_amd.shard import visible_gpu_count
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2")
    assert visible_gpu_count() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")  # HIP's list wins (it indexes into ROCR's)
    assert visible_gpu_count() == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert visible_gpu_count() == 0


@pytest.mark.parametrize("nj,ngpu", [(5, 2), (4, 8), (20, None)])
def test_driver_cmd_branch_spreads_jobs_over_gpus(tmp_path, monkeypatch, nj, ngpu):
    """ngpu None: the recipe's unchanged call (--cmd "$train_cmd" --nj 20, e2e/wsj/run_fdlp_e1.sh:196) on
    an 8-GPU node: the driver counts the visible GPUs itself and spreads the JOBs over all of them."""
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    data = tmp_path / "data" / "dev"
    data.mkdir(parents=True)
    (data / "wav.scp").write_text("".join("u%d /x/u%d.wav\n" % (i, i) for i in range(nj * 2)))
    log = tmp_path / "cmd.log"
    env = dict(os.environ, FAKE_CMD_LOG=str(log))
    gpu_opt = ["--ngpu", str(ngpu)] if ngpu else []
    cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", str(nj)] + gpu_opt + [
           "--cmd", os.path.join(ROOT, "tests", "fakes", "fake_run_pl.sh"), "--write_utt2num_frames", "true",
           str(data), str(tmp_path / "fbank")]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = log.read_text().splitlines()
    assert len(lines) == nj
    ngpu = ngpu or 8
    devices = []
    for n, line in enumerate(lines, 1):
        argv = line.split()[2:]  # drop "python3 <cli>"
        assert argv[1].endswith("melspec_dev.%d" % n)
        assert "--device_rr=%d,%d" % (n, ngpu) in argv
        devices.append(_resolve(argv))
    assert devices == [(n - 1) % ngpu for n in range(1, nj + 1)]
    # the resource request the launcher gets for the JOB array: the reference's --mem 5G
    # (recipes/timit/local_pyspeech/make_FDLPspectrum_feats.sh:92) plus one GPU per JOB
    assert (tmp_path / "cmd.log.opts").read_text().split() == ["--mem", "5G", "--gpu", "1"]


def test_driver_cmd_resource_request_options(tmp_path):
    """--job_mem / --job_gpu change the launcher's request (--job_gpu 0 drops the GPU request); the JOB
    argv is the same either way."""
    data = tmp_path / "data" / "dev"
    data.mkdir(parents=True)
    (data / "wav.scp").write_text("".join("u%d /x/u%d.wav\n" % (i, i) for i in range(4)))
    argvs = []
    for extra, want in ((["--job_mem", "8G"], ["--mem", "8G", "--gpu", "1"]), (["--job_gpu", "0"], ["--mem", "5G"])):
        log = tmp_path / ("cmd%d.log" % len(argvs))
        env = dict(os.environ, FAKE_CMD_LOG=str(log), HIP_VISIBLE_DEVICES="0,1")
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "2"] + extra + [
               "--cmd", os.path.join(ROOT, "tests", "fakes", "fake_run_pl.sh"), str(data), str(tmp_path / "fbank")]
        r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert (tmp_path / (log.name + ".opts")).read_text().split() == want
        argvs.append(log.read_text())
    assert argvs[0] == argvs[1]


def test_native_cli_process_never_imports_torch(tmp_path):
    """A cold compute-fdlp-feats JOB on the native runner (the default) loads libfdlp_hip.so without
    importing torch (about 2 s per process): whatever happens on this host (no GPU here: the JOB fails at
    HIP initialisation; on a GPU box it completes), torch is never imported."""
    import sys
    import numpy as np
    from scipy.io import wavfile
    w = str(tmp_path / "a.wav")
    wavfile.write(w, 16000, (np.random.default_rng(0).standard_normal(32000) * 1000).astype(np.int16))
    scp = tmp_path / "w.scp"
    scp.write_text("u1 %s\n" % w)
    code = ("import sys\n"
            "sys.path.insert(0, %r)\n"
            "from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import main\n"
            "try:\n"
            "    main([%r, %r, '--nfilters=80', '--order=150', '--coeff_num=100', '--coeff_range=0,100',\n"
            "          '--fduration=1.5', '--fbank_type=cochlear,1,1,1,2.5,1', '--seed=1'])\n"
            "    print('RESULT ok')\n"
            "except Exception as e:\n"
            "    print('RESULT', type(e).__name__)\n"
            "print('TORCH', 'torch' in sys.modules)\n") % (ROOT, str(scp), str(tmp_path / "o"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert "TORCH False" in r.stdout, r.stdout + r.stderr
    assert "RESULT" in r.stdout, r.stdout + r.stderr


def test_native_jobs_open_only_their_gpu(monkeypatch):
    """A cold native JOB narrows HIP_VISIBLE_DEVICES to its own GPU before the HIP runtime starts (one device
    initialised instead of every GPU of the node) and addresses it as device 0."""
    from speech_recognition_tools_amd.featgen.computeFDLPSpectrogram import build_parser, narrow_visible_devices
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    env = {}
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    a = narrow_visible_devices(build_parser().parse_args(["a.scp", "o", "--device_rr=11,8"]), env)
    assert env["HIP_VISIBLE_DEVICES"] == "2" and a.device == 0 and a.device_rr is None
    env = {"HIP_VISIBLE_DEVICES": "4,5,6,7"}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5,6,7")
    a = narrow_visible_devices(build_parser().parse_args(["a.scp", "o", "--device_rr=2,4"]), env)
    assert env["HIP_VISIBLE_DEVICES"] == "5" and a.device == 0


FAKE_CLI = r'''
import os, sys
args = [a for a in sys.argv[1:] if not a.startswith("--")]
lst, out = args[0], args[1]
with open(os.environ["FAKE_CLI_LOG"], "a") as f:
    f.write(out + "\n")
utts = [l.split()[0] for l in open(lst) if l.strip()]
open(out + ".ark", "w").write("ark")
open(out + ".scp", "w").write("".join("%s %s.ark:%d\n" % (u, out, i) for i, u in enumerate(utts)))
open(out + ".len", "w").write("".join("%s 1\n" % u for u in utts))
'''


def _resume_setup(tmp_path):
    src = tmp_path / "src" / "featgen"
    src.mkdir(parents=True)
    (src / "computeFDLPSpectrogram.py").write_text(FAKE_CLI)
    data = tmp_path / "data" / "dev"
    data.mkdir(parents=True)
    (data / "wav.scp").write_text("".join("u%d /x/u%d.wav\n" % (i, i) for i in range(9)))
    log = tmp_path / "cli.log"

    def run(*extra):
        if log.exists():
            log.unlink()
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "3", "--ngpu", "1",
               "--src_dir", str(tmp_path / "src"), "--write_utt2num_frames", "true"] + list(extra) + [
               str(data), str(tmp_path / "fbank")]
        r = subprocess.run(cmd, cwd=str(tmp_path), env=dict(os.environ, FAKE_CLI_LOG=str(log)),
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        ran = sorted(int(l.rsplit(".", 1)[1]) for l in log.read_text().split()) if log.exists() else []
        assert len((data / "feats.scp").read_text().splitlines()) == 9
        assert len((data / "utt2num_frames").read_text().splitlines()) == 9
        return ran
    return run, tmp_path / "fbank"


def test_driver_resume_skips_finished_jobs(tmp_path):
    """--resume true (SURVEY.md §5 checkpoint/resume row): a rerun skips the JOBs whose last finished run
    had the same shard and options and whose ark/scp exist; a JOB whose output went missing, or a change of
    the feature options, reruns; without --resume every JOB runs as in the reference driver."""
    run, fbank = _resume_setup(tmp_path)
    assert run() == [1, 2, 3]
    assert all((fbank / ("melspec_dev.%d.done" % n)).exists() for n in (1, 2, 3))
    assert run("--resume", "true") == []
    (fbank / "melspec_dev.2.ark").unlink()
    assert run("--resume", "true") == [2]
    assert run("--resume", "true", "--order", "40") == [1, 2, 3]  # other options: new keys
    assert run("--resume", "true", "--order", "40") == []
    assert run() == [1, 2, 3]
    (fbank / "melspec_dev.3.len").unlink()  # --write_utt2num_frames: the .len is an output too
    assert run("--resume", "true") == [3]


def test_driver_resume_sees_edits_of_the_files_the_options_name(tmp_path):
    """The resume key hashes the contents of the files the options name: an in-place edit
    of the --lifter_config file reruns every JOB with the same option string."""
    run, fbank = _resume_setup(tmp_path)
    lif = tmp_path / "lifter.txt"
    lif.write_text("1.0 " * 100 + "\n")
    assert run("--lifter_config", str(lif)) == [1, 2, 3]
    assert run("--resume", "true", "--lifter_config", str(lif)) == []
    lif.write_text("0.5 " * 100 + "\n")
    assert run("--resume", "true", "--lifter_config", str(lif)) == [1, 2, 3]


def test_driver_resume_with_launcher_wraps_jobs_in_the_guard(tmp_path):
    """With a $cmd launcher the JOB array is still launched whole (JOB=1:n is a range) and every JOB runs
    behind scripts/fdlp_resume_guard.sh; the command after the guard's "--" is the unguarded JOB argv."""
    data = tmp_path / "data" / "dev"
    data.mkdir(parents=True)
    (data / "wav.scp").write_text("".join("u%d /x/u%d.wav\n" % (i, i) for i in range(4)))
    logs = []
    for extra in ([], ["--resume", "true"]):
        log = tmp_path / ("cmd%d.log" % len(logs))
        env = dict(os.environ, FAKE_CMD_LOG=str(log), HIP_VISIBLE_DEVICES="0,1")
        cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "2"] + extra + [
               "--cmd", os.path.join(ROOT, "tests", "fakes", "fake_run_pl.sh"), str(data), str(tmp_path / "fbank")]
        r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        logs.append(log.read_text().splitlines())
    for plain, guarded in zip(*logs):
        g = guarded.split()
        assert g[0] == "bash" and g[1].endswith("fdlp_resume_guard.sh")
        assert " ".join(g[g.index("--") + 1:]) == plain


def test_resume_guard(tmp_path):
    guard = os.path.join(ROOT, "scripts", "fdlp_resume_guard.sh")
    key, stamp, out = tmp_path / "k", tmp_path / "s", tmp_path / "o"
    key.write_text("1 2\n")
    mark = tmp_path / "ran"

    def go(*command):
        if mark.exists():
            mark.unlink()
        r = subprocess.run(["bash", guard, str(key), str(stamp), str(out), "--"] + list(command),
                           capture_output=True, text=True, timeout=60)
        return r.returncode, mark.exists()
    assert go("false") == (1, False) and not stamp.exists()  # a failed JOB leaves no stamp
    assert go("touch", str(mark)) == (0, True) and stamp.read_text() == "1 2\n"
    assert go("touch", str(mark)) == (0, True)  # stamp matches but no outputs yet: runs
    (tmp_path / "o.ark").write_text("")
    (tmp_path / "o.scp").write_text("")
    assert go("touch", str(mark)) == (0, False)  # up to date: skipped
    key.write_text("3 4\n")
    assert go("touch", str(mark)) == (0, True) and stamp.read_text() == "3 4\n"
    # extra outputs before the "--" (.len, CMVN stats): all must exist for a skip
    extra = tmp_path / "o.len"
    r = subprocess.run(["bash", guard, str(key), str(stamp), str(out), str(extra), "--", "touch", str(mark)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and mark.exists()
    mark.unlink()
    extra.write_text("")
    r = subprocess.run(["bash", guard, str(key), str(stamp), str(out), str(extra), "--", "touch", str(mark)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and not mark.exists()


def test_early_hip_start_narrows_like_main(monkeypatch):
    """A cold JOB parses its argv with the real parser before numpy is imported (featgen/_early_hip.py):
    the native runner's GPU becomes the only visible one exactly as main() would narrow it, main() then
    addresses it as device 0, and the python runner / --add_reverb leave the environment alone."""
    import sys
    from speech_recognition_tools_amd.featgen import _early_hip
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setattr(_early_hip, "NARROWED", False)
    monkeypatch.setattr(_early_hip, "_thread", None)
    monkeypatch.setattr(_early_hip, "_warm", lambda dev: None)  # no HIP runtime start in the CPU suite
    had_torch = sys.modules.pop("torch", None)
    try:
        for argv in (["a.scp", "o", "--host_runner=python"], ["a.scp", "o", "--add_reverb=small_room"]):
            _early_hip.start(argv)
            assert not _early_hip.NARROWED and "HIP_VISIBLE_DEVICES" not in os.environ
        monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1,2,3")
        _early_hip.start(["a.scp", "o", "--device_rr=3,4"])
        assert _early_hip.NARROWED and os.environ["HIP_VISIBLE_DEVICES"] == "2"
        _early_hip.join()
    finally:
        if had_torch is not None:
            sys.modules["torch"] = had_torch
        monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)


def test_early_hip_warms_the_jobs_own_device(monkeypatch):
    """ADVICE r5 / VERDICT r5 item 8: with CUDA_VISIBLE_DEVICES set the visible set is not narrowed, and the
    helper must warm the GPU main() will use (resolve_device), not device 0; unknown options start nothing
    (main()'s parse_args exits 2 with no helper inside the HIP runtime start)."""
    import sys
    from speech_recognition_tools_amd.featgen import _early_hip
    for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    had_torch = sys.modules.pop("torch", None)
    warmed = []
    monkeypatch.setattr(_early_hip, "_warm", lambda dev: warmed.append(dev))
    monkeypatch.setattr(_early_hip, "NARROWED", False)
    monkeypatch.setattr(_early_hip, "_thread", None)
    try:
        assert _early_hip.warm_target(["a.scp", "o", "--device_rr", "3,4"]) == (2, False)
        assert _early_hip.warm_target(["a.scp", "o", "--device", "5"]) == (5, False)
        assert _early_hip.warm_target(["a.scp", "o", "--bogus_option"]) is None
        assert _early_hip.warm_target(["a.scp", "o", "--device_rr", "0,4"]) is None  # main() raises it
        _early_hip.start(["a.scp", "o", "--device_rr", "3,4"])
        _early_hip.join()
        assert warmed == [2] and not _early_hip.NARROWED and "HIP_VISIBLE_DEVICES" not in os.environ
    finally:
        if had_torch is not None:
            sys.modules["torch"] = had_torch


def test_cli_unknown_option_exits_2_cleanly(tmp_path):
    """A misspelled option: usage error, exit status 2, and no HIP helper was started."""
    cli = os.path.join(ROOT, "bin", "compute-fdlp-feats")
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    r = subprocess.run(["bash", cli, "a.scp", str(tmp_path / "o"), "--no_such_option"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "unrecognized arguments" in r.stderr


CHAIN_CLI = r'''
import os, sys
args = [a for a in sys.argv[1:] if not a.startswith("--")]
lst, out = args[0], args[1]
print("job", out, "pid", os.getpid(), "keep_warm", "--keep_warm" in sys.argv)
with open(os.environ["FAKE_CLI_LOG"], "a") as f:
    f.write("%s %d\n" % (out, os.getpid()))
if out.endswith(".4") and os.environ.get("FAIL_JOB4"):
    raise RuntimeError("JOB 4 fails")
utts = [l.split()[0] for l in open(lst) if l.strip()]
open(out + ".ark", "w").write("ark")
open(out + ".scp", "w").write("".join("%s %s.ark:%d\n" % (u, out, i) for i, u in enumerate(utts)))
open(out + ".len", "w").write("".join("%s 1\n" % u for u in utts))
'''


@pytest.mark.parametrize("fail", [False, True])
def test_driver_chains_run_jobs_in_warm_processes(tmp_path, fail):
    """Without $cmd the driver's N*K slots are JOB chains (featgen/job_chain.py): 7 JOBs on 2 GPUs at 2 per
    GPU run in 4 processes, each chain's JOBs on one GPU, every JOB with its own log, outputs and done
    stamp and with --keep_warm; a failing JOB fails the driver but not the rest of its chain."""
    src = tmp_path / "src" / "featgen"
    src.mkdir(parents=True)
    (src / "computeFDLPSpectrogram.py").write_text(CHAIN_CLI)
    data = tmp_path / "data" / "dev"
    data.mkdir(parents=True)
    (data / "wav.scp").write_text("".join("u%d /x/u%d.wav\n" % (i, i) for i in range(14)))
    log = tmp_path / "cli.log"
    env = dict(os.environ, FAKE_CLI_LOG=str(log))
    if fail:
        env["FAIL_JOB4"] = "1"
    cmd = ["bash", os.path.join(ROOT, "scripts", "make_FDLPspectrum_feats.sh"), "--nj", "7", "--ngpu", "2",
           "--jobs_per_gpu", "2", "--src_dir", str(tmp_path / "src"), "--write_utt2num_frames", "true",
           str(data), str(tmp_path / "fbank")]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=120)
    ran = [l.split() for l in log.read_text().splitlines()]
    assert sorted(int(o.rsplit(".", 1)[1]) for o, _ in ran) == list(range(1, 8))
    pids = {}
    for o, pid in ran:
        pids.setdefault(pid, []).append(int(o.rsplit(".", 1)[1]))
    assert len(pids) == 4
    for jobs in pids.values():  # one GPU per chain: JOB n on GPU (n - 1) mod 2
        assert len({(n - 1) % 2 for n in jobs}) == 1
    for n in range(1, 8):
        text = (data / "log" / ("feats_dev.%d.log" % n)).read_text()
        assert ("melspec_dev.%d " % n) in text and "keep_warm True" in text
        assert (tmp_path / "fbank" / ("melspec_dev.%d.done" % n)).exists() == (not (fail and n == 4))
    if fail:
        assert r.returncode != 0
        assert "JOB 4 fails" in (data / "log" / "feats_dev.4.log").read_text()
    else:
        assert r.returncode == 0, r.stdout + r.stderr
        assert len((data / "feats.scp").read_text().splitlines()) == 14
