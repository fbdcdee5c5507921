#!/usr/bin/env bash
# Stand-in for Kaldi's utils/run.pl in driver tests: fake_run_pl.sh JOB=a:b <log> <command...>
# records every JOB's command line (JOB substituted) in $FAKE_CMD_LOG and creates the per-JOB files
# make_FDLPspectrum_feats.sh concatenates (<outfile>.scp / .len), without running the command.
# Kaldi launchers take "--opt value" pairs before JOB=a:b (run.pl ignores them, queue.pl / slurm.pl map
# --mem / --gpu to the scheduler); they are recorded in $FAKE_CMD_LOG.opts.
opts=()
while [[ "$1" == --* ]]; do opts+=("$1" "$2"); shift 2; done
[ -n "${FAKE_CMD_LOG:-}" ] && printf '%s\n' "${opts[*]}" >> "$FAKE_CMD_LOG.opts"
range=${1#JOB=}; shift
shift  # log file
for n in $(seq "${range%%:*}" "${range##*:}"); do
  args=()
  for a in "$@"; do args+=("${a//JOB/$n}"); done
  printf '%s\n' "${args[*]}" >> "$FAKE_CMD_LOG"
  for i in "${!args[@]}"; do  # the output prefix follows "<cli>.py <list>"
    [[ "${args[$i]}" == *.py ]] && { touch "${args[$((i + 2))]}.scp" "${args[$((i + 2))]}.len"; break; }
  done
done
