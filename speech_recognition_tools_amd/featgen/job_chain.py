#!/usr/bin/env python3
"""Run several JOBs of make_FDLPspectrum_feats.sh in one warm process (the driver's JOB chains).

The reference driver starts one cold `computeFDLPSpectrogram.py` process per JOB
(recipes/timit/local_pyspeech/make_FDLPspectrum_feats.sh:141-157, `$cmd JOB=1:$nj`).  On an MI355X a JOB's
device work is milliseconds, so at the recipes' --nj 20 a cold process's fixed costs -- interpreter and
imports, the HIP runtime start, the plan build, page-locking its slots -- are most of stage 1
(profiles/r06e_driver_e2e.jsonl: 20 cold JOBs over 10 audio-hours on one GPU 5.1 s, the same data as one
JOB 0.8 s).  A chain runs its JOBs one after the other in one process with --keep_warm, so only the first
pays them; each JOB still reads its own shard and writes its own <outfile>.ark/.scp/.len, its log goes to
its own log file (stdout and stderr of the process, the native runner's included, are pointed at it while
the JOB runs) and a JOB that fails does not stop the chain.

    job_chain.py --jobs 1,5,9 --log LOG_PATTERN [--key KEY_PATTERN --done DONE_PATTERN] [--cli PATH] -- CLI_ARGS...

Every "JOB" in the patterns and in CLI_ARGS is replaced by the JOB's number (as run.pl / queue.pl do).  After
a JOB succeeds its key file is copied to its done file (the driver's --resume stamp).  Exit status 1 if any
JOB failed.  The chain's JOBs must run on one GPU (the driver groups them by --device_rr).  --cli (default:
this package's computeFDLPSpectrogram.py, the driver's --src_dir one otherwise) runs as its own process
would run it: as __main__, with sys.argv = [cli] + the JOB's arguments.
"""
import os
import runpy
import shutil
import sys
import traceback

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CLI = os.path.join(os.path.dirname(os.path.abspath(__file__)), "computeFDLPSpectrogram.py")


def _parse(argv):
    if "--" not in argv:
        raise SystemExit("usage: job_chain.py --jobs N[,N...] --log PATTERN [--key P --done P] -- CLI_ARGS")
    i = argv.index("--")
    head, cli = argv[:i], argv[i + 1:]
    opts = {"--jobs": None, "--log": None, "--key": None, "--done": None, "--cli": CLI}
    k = 0
    while k < len(head):
        if head[k] not in opts or k + 1 >= len(head):
            raise SystemExit("job_chain.py: unknown or incomplete option %r" % head[k])
        opts[head[k]] = head[k + 1]
        k += 2
    if not opts["--jobs"] or not opts["--log"]:
        raise SystemExit("job_chain.py: --jobs and --log are required")
    jobs = [int(j) for j in opts["--jobs"].split(",") if j.strip()]
    return jobs, opts["--log"], opts["--key"], opts["--done"], opts["--cli"], cli


def _libc_flush():
    try:
        import ctypes
        ctypes.CDLL(None).fflush(None)
    except (OSError, AttributeError):
        pass


def _sub(s, n):
    return s.replace("JOB", str(n))


def main(argv=None):
    jobs, log_pat, key_pat, done_pat, cli_path, cli = _parse(sys.argv[1:] if argv is None else argv)
    if not jobs:
        return 0
    first = [_sub(a, jobs[0]) for a in cli]
    from speech_recognition_tools_amd.featgen import _early_hip
    _early_hip.start(first)  # the HIP runtime starts while the CLI imports numpy (its own start() then returns)
    failed = 0
    saved = (os.dup(1), os.dup(2))
    try:
        for n in jobs:
            args = [_sub(a, n) for a in cli]
            if "--keep_warm" not in args:
                args.append("--keep_warm")
            sys.stdout.flush()
            sys.stderr.flush()
            with open(_sub(log_pat, n), "w") as log:
                os.dup2(log.fileno(), 1)
                os.dup2(log.fileno(), 2)
                sys.argv = [cli_path] + args
                ok = False
                try:
                    runpy.run_path(cli_path, run_name="__main__")
                    ok = True
                except SystemExit as e:  # a usage error: the CLI printed it
                    ok = e.code in (None, 0)
                except BaseException:  # the JOB's exception, as its own process would print it
                    traceback.print_exc()
                sys.stdout.flush()
                sys.stderr.flush()
                _libc_flush()  # the native runner's progress lines (C stdio) belong to this JOB's log
                os.dup2(saved[0], 1)
                os.dup2(saved[1], 2)
            if ok and key_pat and done_pat:
                shutil.copyfile(_sub(key_pat, n), _sub(done_pat, n))
            if not ok:
                failed += 1
                sys.stderr.write("job_chain.py: JOB %d failed, see %s\n" % (n, _sub(log_pat, n)))
    finally:
        os.dup2(saved[0], 1)
        os.dup2(saved[1], 2)
        os.close(saved[0])
        os.close(saved[1])
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
