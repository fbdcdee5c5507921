#!/usr/bin/env bash
# Stand-in for Kaldi's utils/run.pl in driver tests: fake_run_pl.sh JOB=a:b <log> <command...>
# records every JOB's command line (JOB substituted) in $FAKE_CMD_LOG and creates the per-JOB files
# make_FDLPspectrum_feats.sh concatenates (<outfile>.scp / .len), without running the command.
range=${1#JOB=}; shift
shift  # log file
for n in $(seq "${range%%:*}" "${range##*:}"); do
  args=()
  for a in "$@"; do args+=("${a//JOB/$n}"); done
  printf '%s\n' "${args[*]}" >> "$FAKE_CMD_LOG"
  touch "${args[3]}.scp" "${args[3]}.len"
done
