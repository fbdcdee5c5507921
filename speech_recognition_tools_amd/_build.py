"""Build libfdlp_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libfdlp_hip.so")
SOURCES = ["fdlp_dct.hip", "fdlp_autocorr.hip", "fdlp_lpc.hip", "fdlp_misc.hip", "fdlp_plan.cpp", "fdlp_host.cpp",
           "fdlp_job.cpp"]
HEADERS = ["fdlp_internal.h", "fdlp_device.h", "fdlp_error.h", os.path.join("..", "..", "include", "fdlp.h")]
ARCH = os.environ.get("FDLP_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return False


def build(force=False, verbose=False, out=None, defines=()):
    """out / defines: an A/B variant of the library (e.g. -DFDLP_DEVICE_CHECKS=1) at another path, loaded
    through FDLP_LIB; the default build is LIB."""
    target = out or LIB
    if not force and out is None and not stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)
    objs, cmds = [], []
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function",
             "-munsafe-fp-atomics"] + list(defines)
    tag = "." + os.path.basename(target).replace(".", "_") if out else ""
    for src in SOURCES:
        obj = os.path.join(LIBDIR, src + tag + ".o")
        lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "c++"]
        cmd = [hipcc()] + flags + lang + ["-c", os.path.join(CSRC, src), "-o", obj]
        if src.endswith(".cpp"):
            cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-Wall",
                   "-x", "c++", "-c", os.path.join(CSRC, src), "-o", obj] + [d for d in defines if d.startswith("-D")]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        cmds.append(cmd)
        objs.append(obj)
    # the translation units compile in parallel, at most one per host CPU; every started compiler is
    # waited for (subprocess.run), and the first failure is raised after all have finished
    from concurrent.futures import ThreadPoolExecutor
    workers = max(1, min(len(cmds), os.cpu_count() or 1))
    with ThreadPoolExecutor(max_workers=workers) as pool:
        rcs = list(pool.map(lambda c: subprocess.run(c).returncode, cmds))
    failed = [c for c, rc in zip(cmds, rcs) if rc != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    tmp = target + ".tmp"
    cmd = [hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    for o in objs:
        os.unlink(o)
    return target


if __name__ == "__main__":
    # python _build.py [--force] [--out PATH -DNAME=VALUE ...]
    argv = sys.argv[1:]
    out = argv[argv.index("--out") + 1] if "--out" in argv else None
    defs = [a for a in argv if a.startswith("-D")]
    print(build(force="--force" in argv, verbose=True, out=out, defines=defs))
