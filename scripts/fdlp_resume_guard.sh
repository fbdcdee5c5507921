#!/usr/bin/env bash
# Per-JOB resume guard of make_FDLPspectrum_feats.sh --resume true:
#   fdlp_resume_guard.sh <key> <stamp> <output-prefix> [<extra output> ...] -- <command...>
# <key> holds the JOB's identity (a hash of its shard, the feature options and the files they name),
# <stamp> the key of the last run of this JOB that finished.  When they match and the JOB's outputs
# (<output-prefix>.ark/.scp and every extra output: the .len, the CMVN stats) exist, the JOB is skipped;
# otherwise the command runs (as a child) and, if it succeeds, the key is copied to the stamp.  The outputs
# themselves are published atomically by the CLI (tmp + rename), so a stamp never names a half-written ark.
key=$1 stamp=$2 out=$3
shift 3
extra=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do extra+=("$1"); shift; done
[ "$1" = "--" ] && shift
have_all() { local f; for f in "$out.ark" "$out.scp" "${extra[@]}"; do [ -f "$f" ] || return 1; done; }
if [ -s "$key" ] && cmp -s "$key" "$stamp" && have_all; then
  echo "$0: $out is up to date (resume), skipped"
  exit 0
fi
rm -f "$stamp"
"$@"
rc=$?
[ $rc -eq 0 ] && cp "$key" "$stamp"
exit $rc
