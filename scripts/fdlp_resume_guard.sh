#!/usr/bin/env bash
# Per-JOB resume guard of make_FDLPspectrum_feats.sh --resume true:
#   fdlp_resume_guard.sh <key> <stamp> <output-prefix> -- <command...>
# <key> holds the JOB's identity (a hash of its shard and the feature options), <stamp> the key of the
# last run of this JOB that finished.  When they match and the JOB's outputs (<output-prefix>.ark/.scp)
# exist, the JOB is skipped; otherwise the command runs (as a child) and, if it succeeds, the key is
# copied to the stamp.  The outputs themselves are published atomically by the CLI (tmp + rename), so a
# stamp never names a half-written ark.
key=$1 stamp=$2 out=$3
shift 3
[ "$1" = "--" ] && shift
if [ -s "$key" ] && cmp -s "$key" "$stamp" && [ -f "$out.ark" ] && [ -f "$out.scp" ]; then
  echo "$0: $out is up to date (resume), skipped"
  exit 0
fi
rm -f "$stamp"
"$@"
rc=$?
[ $rc -eq 0 ] && cp "$key" "$stamp"
exit $rc
