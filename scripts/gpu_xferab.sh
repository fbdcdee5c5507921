set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r05zf; mkdir -p $O; : > $O/ab.txt
for round in 1 2; do
  for n in A D hip; do
    FDLP_LIB=$PWD/speech_recognition_tools_amd/lib/libfdlp_$n.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --xfer-variants "" > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 3; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); t=d.get('with_transfers') or {}
print(sys.argv[1], round(d['value'],1), 'xfer', round(t.get('value',0) or 0,1))" $n $O/run.log >> $O/ab.txt
  done
done
cat $O/ab.txt
