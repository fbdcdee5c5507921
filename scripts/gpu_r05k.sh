set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
for j in 2 4 8; do
timeout -k 10 300 python -u benchmarks/driver_e2e.py --utts 1800 --nj 8 --jobs-per-gpu $j > $O/driver_j$j.json 2> $O/driver_j$j.err || { tail -20 $O/driver_j$j.err; exit 1; }
python3 -c "
import json; r=json.load(open('$O/driver_j$j.json')); print($j, round(r['value'],3), round(r['wall_s'],3), r['job_execution_s'], r['one_cold_job'])"
done
