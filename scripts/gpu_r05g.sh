set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_ola.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ARGS="--ola-path separate|--ola-path fused" TAG=r05g TRACE=1 bash scripts/gpu_ab.sh || exit 2
python3 - <<'PY'
import csv
for v in ("separate", "fused"):
    for r in csv.DictReader(open("gpurun_out/r05g/trace___ola_path_%s_.csv" % v)):
        if "lattice" in r["kernel"] or "ola" in r["kernel"]: print(v, r["kernel"].split("(")[0][-45:], r["avg_ms"])
PY
