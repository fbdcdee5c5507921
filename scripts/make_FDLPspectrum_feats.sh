#!/usr/bin/env bash
# Drop-in for recipes/timit/local_pyspeech/make_FDLPspectrum_feats.sh of
# sadhusamik/speech_recognition_tools (same options and outputs), running each JOB's
# compute-fdlp-feats on an MI355X.  Extra options: --ngpu N (JOB n runs on GPU (n-1) mod N, with or
# without a Kaldi $cmd launcher: the CLI gets --device_rr=JOB,N and picks the device before any GPU
# call, folded into the GPUs that JOB can see; default: every visible GPU, counted without touching
# HIP -- HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES if set, else the KFD
# topology's GPU nodes -- so a recipe that calls the driver unchanged, e.g. --cmd "$train_cmd" --nj 20
# (e2e/wsj/run_fdlp_e1.sh:196), spreads its JOBs over the node), --jobs_per_gpu K (without $cmd: at most
# N*K JOBs run at once; default 4), --chain_jobs (without $cmd, default true: those N*K slots are warm
# processes running their JOBs in turn, featgen/job_chain.py), --job_mem / --job_gpu (the resource request a $cmd launcher gets for
# every JOB: "$cmd --mem 5G --gpu 1 JOB=1:$nj ...", the reference's --mem 5G (:92, :141) plus one GPU, so
# queue.pl / slurm.pl allocate the MI355X the JOB runs on; run.pl ignores both; --job_gpu 0 drops it),
# --resume true (per-JOB resume: every JOB that finishes leaves <feat_dir>/melspec_<name>.JOB.done holding
# a hash of its shard and the feature options; a rerun with --resume true skips the JOBs whose stamp
# matches and whose ark/scp exist, through scripts/fdlp_resume_guard.sh, and reruns the rest; the
# concatenated feats.scp / utt2num_frames are rebuilt from every JOB's files as usual).
#
#   make_FDLPspectrum_feats.sh [--opts] <data_dir> <feat_dir>
# Inputs: <data_dir>/wav.scp or <data_dir>/segments.  Outputs: <data_dir>/feats.scp,
# <data_dir>/utt2num_frames (with --write_utt2num_frames true), <feat_dir>/melspec_<name>.JOB.{ark,scp,len}.

[ -f ./path.sh ] && . ./path.sh

nj=100
nfilters=20
fduration=0.5
coeff_num=50
coeff_range='0,30'
order=50
overlap_fraction=0.25
add_reverb=clean
add_noise=clean
fbank_type="mel,1"
gamma_weight="None"
odd_mod_zero=false
frate=100
cmd=
add_opts=
src_dir=
spectrum_type=log
write_utt2num_frames=false
lifter_config=
check_for_segment="data/train"
ngpu=          # default: the visible GPU count (visible_gpus below)
jobs_per_gpu=4  # JOBs per GPU at once: their kernels overlap on the device and the cold
               # processes' fixed costs (interpreter, HIP runtime start) overlap each other: 8 cold JOBs on
               # one GPU 0.71 / 1.03 / 1.09 audio-h/s at 2 / 4 / 8 (profiles/r05k_driver_jobs_per_gpu.jsonl)
compute_cmvn=false   # also write <data_dir>/cmvn.ark (global CMVN stats, fused on the device)
seed=
noise_seed=
job_mem=5G     # $cmd --mem (the reference driver's request, make_FDLPspectrum_feats.sh:92, :141)
job_gpu=1      # $cmd --gpu (0: no GPU request)
resume=false   # skip JOBs whose last finished run had the same shard and options (and whose outputs exist)
chain_jobs=true  # without $cmd: the N*K concurrent slots are warm processes that run their JOBs one after the
                 # other (featgen/job_chain.py: each JOB's own shard, outputs and log), so only a slot's first
                 # JOB pays the cold start; false: one cold process per JOB, as the reference driver

if [ -f utils/parse_options.sh ]; then
  . utils/parse_options.sh || exit 1
else
  while [ $# -gt 0 ]; do
    case "$1" in
      --*=*) k="${1%%=*}"; k="${k#--}"; v="${1#*=}"; shift ;;
      --*) k="${1#--}"; v="$2"; shift 2 ;;
      *) break ;;
    esac
    k="${k//-/_}"
    eval "$k=\"\$v\""
  done
fi

visible_gpus() {  # GPUs this process may use, without initialising HIP
  local v n=0 f id
  for v in HIP_VISIBLE_DEVICES ROCR_VISIBLE_DEVICES CUDA_VISIBLE_DEVICES; do
    if [ -n "${!v+x}" ]; then
      IFS=, read -ra ids <<< "${!v}"
      for id in "${ids[@]}"; do [ -n "${id// /}" ] && n=$((n + 1)); done
      echo $n; return
    fi
  done
  for f in /sys/class/kfd/kfd/topology/nodes/*/gpu_id; do
    [ -r "$f" ] && read -r id < "$f" && [ "${id:-0}" != 0 ] && n=$((n + 1))
  done
  echo $n
}
[ -z "$ngpu" ] && ngpu=$(visible_gpus)
[ "${ngpu:-0}" -ge 1 ] 2>/dev/null || ngpu=1

here="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
[ -z "$src_dir" ] && src_dir="$here/speech_recognition_tools_amd"
cli="$src_dir/featgen/computeFDLPSpectrogram.py"

if [ $# -ne 2 ]; then
  echo "Usage: $0 [--opts] <data_dir> <feat_dir>"; exit 1
fi
data_dir=$1
feat_dir=$2
echo "$0 $@"
case "$feat_dir" in /*) ;; *) feat_dir="$PWD/$feat_dir" ;; esac
mkdir -p "$feat_dir"

name=$(basename "$data_dir")
scp=$data_dir/wav.scp
segment=$data_dir/segments
log_dir=$data_dir/log
mkdir -p "$log_dir"

$odd_mod_zero && add_opts="$add_opts --odd_mod_zero"
$write_utt2num_frames && add_opts="$add_opts --write_utt2num_frames"
[ -n "$lifter_config" ] && add_opts="$add_opts --lifter_config $lifter_config"
[ -n "$seed" ] && add_opts="$add_opts --seed $seed"
[ -n "$noise_seed" ] && add_opts="$add_opts --noise_seed $noise_seed"

split_list() {  # split_list <in> <out1> ... : contiguous, balanced, like utils/split_scp.pl
  local in=$1; shift
  if [ -f utils/split_scp.pl ]; then utils/split_scp.pl "$in" "$@"; return $?; fi
  python3 "$here/speech_recognition_tools_amd/shard.py" "$in" "$@"
}

feat_opts="--fbank_type=$fbank_type --gamma_weight=$gamma_weight --add_reverb=$add_reverb \
--add_noise=$add_noise --coeff_num=$coeff_num --coeff_range=$coeff_range --order=$order \
--overlap_fraction=$overlap_fraction --nfilters=$nfilters --fduration=$fduration --frate=$frate"

# the files the options name, whose contents the features depend on (an in-place edit must invalidate a
# finished JOB): --lifter_config, noises/<type>.wav of --add_noise <type>,<snr> and the RIR of --add_reverb
# (both relative to the working directory, features.py:34-44, :75-91), and wav.scp + segments when the
# shards are segment dumps (their scp lines are ark offsets, unchanged by an edit of the audio)
ref_files=()
[ -n "$lifter_config" ] && ref_files+=("$lifter_config")
case $add_noise in clean|diff) ;; *) ref_files+=("noises/${add_noise%%,*}.wav") ;; esac
case $add_reverb in
  small_room) ref_files+=(./RIR/RIR_SmallRoom1_near_AnglA.wav) ;;
  medium_room) ref_files+=(./RIR/RIR_MediumRoom1_far_AnglA.wav) ;;
  large_room) ref_files+=(./RIR/RIR_LargeRoom1_far_AnglA.wav) ;;
esac
[ -f "$segment" ] && ref_files+=("$scp" "$segment")
ref_sums() { local f; for f in "${ref_files[@]}"; do echo "$f $(cksum < "$f" 2>/dev/null || echo missing)"; done; }

job_key() {  # job_key <n> <shard> <scp-type-opt>: the JOB's identity, written to its key file
  local n=$1 shard=$2 stype=$3
  { echo "$add_opts $stype $feat_opts compute_cmvn=$compute_cmvn"; ref_sums; cat "$shard"; } | cksum \
    > "$log_dir/resume_${name}.$n.key"
}
job_outputs() {  # job_outputs <n>: every output a finished JOB leaves (the .len and CMVN stats when asked for)
  local out="$feat_dir/melspec_${name}.$1"
  echo "$out.ark" "$out.scp"
  $write_utt2num_frames && echo "$out.len"
  $compute_cmvn && echo "$feat_dir/cmvn_${name}.$1.mat"
}
job_done() {  # the JOB's last finished run had the same key and all its outputs exist
  local n=$1 f
  cmp -s "$log_dir/resume_${name}.$n.key" "$feat_dir/melspec_${name}.$n.done" || return 1
  for f in $(job_outputs $n); do [ -f "$f" ] || return 1; done
}

run_jobs() {  # run_jobs <list-pattern containing JOB> <scp-type-opt>
  local pattern=$1 stype=$2
  local cmvn_opt= n pending=()
  $compute_cmvn && cmvn_opt="--cmvn_stats $feat_dir/cmvn_${name}.JOB.mat"
  for n in $(seq $nj); do
    job_key $n "${pattern//JOB/$n}" "$stype"
    if $resume && job_done $n; then
      echo "$0: JOB $n is up to date (--resume true), skipped"
    else
      rm -f "$feat_dir/melspec_${name}.$n.done"
      pending+=($n)
    fi
  done
  [ ${#pending[@]} -eq 0 ] && return 0
  if [ -n "$cmd" ]; then
    local req= guard=()
    [ -n "$job_mem" ] && req="--mem $job_mem"
    [ "${job_gpu:-0}" != 0 ] && req="$req --gpu $job_gpu"
    # with --resume the launcher still gets the whole JOB array (JOB=a:b is a range); the guard skips
    # the finished JOBs inside it
    local extra_out=()
    $write_utt2num_frames && extra_out+=("$feat_dir/melspec_${name}.JOB.len")
    $compute_cmvn && extra_out+=("$feat_dir/cmvn_${name}.JOB.mat")
    $resume && guard=(bash "$here/scripts/fdlp_resume_guard.sh" "$log_dir/resume_${name}.JOB.key"
                      "$feat_dir/melspec_${name}.JOB.done" "$feat_dir/melspec_${name}.JOB" "${extra_out[@]}" --)
    $cmd $req JOB=1:$nj "$log_dir/feats_${name}.JOB.log" \
      "${guard[@]}" python3 "$cli" "$pattern" "$feat_dir/melspec_${name}.JOB" $add_opts $cmvn_opt $stype \
        --device_rr=JOB,$ngpu $feat_opts || exit 1
    $resume || for n in $(seq $nj); do cp "$log_dir/resume_${name}.$n.key" "$feat_dir/melspec_${name}.$n.done"; done
    return 0
  fi
  local pids=() jobs=() fail=0
  if $chain_jobs; then
    # slots per GPU: JOB n runs on GPU (n-1) mod ngpu (--device_rr), so each chain holds JOBs of one GPU
    local d s k nslot=() chains=()
    for n in "${pending[@]}"; do
      d=$(( (n - 1) % ngpu ))
      k=${nslot[$d]:-0}
      s=$(( d * jobs_per_gpu + k % jobs_per_gpu ))
      chains[$s]="${chains[$s]:+${chains[$s]},}$n"
      nslot[$d]=$(( k + 1 ))
    done
    for s in "${!chains[@]}"; do
      python3 "$here/speech_recognition_tools_amd/featgen/job_chain.py" --jobs "${chains[$s]}" \
        --log "$log_dir/feats_${name}.JOB.log" --key "$log_dir/resume_${name}.JOB.key" \
        --done "$feat_dir/melspec_${name}.JOB.done" --cli "$cli" -- \
        "$pattern" "$feat_dir/melspec_${name}.JOB" $add_opts $cmvn_opt $stype --device_rr=JOB,$ngpu $feat_opts \
        > "$log_dir/chain_${name}.$s.log" 2>&1 &
      pids+=($!)
    done
    for s in "${!pids[@]}"; do wait "${pids[$s]}" || fail=1; done
    [ $fail -eq 0 ] || { echo "$0: a JOB failed, see $log_dir/feats_${name}.*.log"; exit 1; }
    return 0
  fi
  for n in "${pending[@]}"; do
    python3 "$cli" "${pattern//JOB/$n}" "$feat_dir/melspec_${name}.$n" $add_opts ${cmvn_opt//JOB/$n} $stype \
      --device_rr=$n,$ngpu $feat_opts > "$log_dir/feats_${name}.$n.log" 2>&1 &
    pids+=($!)
    jobs+=($n)
    if [ ${#pids[@]} -ge $(( ngpu * jobs_per_gpu )) ]; then
      if wait "${pids[0]}"; then cp "$log_dir/resume_${name}.${jobs[0]}.key" "$feat_dir/melspec_${name}.${jobs[0]}.done"
      else fail=1; fi
      pids=("${pids[@]:1}")
      jobs=("${jobs[@]:1}")
    fi
  done
  local i
  for i in "${!pids[@]}"; do
    if wait "${pids[$i]}"; then cp "$log_dir/resume_${name}.${jobs[$i]}.key" "$feat_dir/melspec_${name}.${jobs[$i]}.done"
    else fail=1; fi
  done
  [ $fail -eq 0 ] || { echo "$0: a JOB failed, see $log_dir/feats_${name}.*.log"; exit 1; }
}

if [ -f "$segment" ]; then
  name_check=$(basename "$check_for_segment")
  if [ -f "$check_for_segment/log/segment_dump/${name_check}_segmentdump.ark" ]; then
    scp_dump_name=$check_for_segment/log/segment_dump/${name_check}_segmentdump
  else
    scp_dump_name=$log_dir/segment_dump/${name}_segmentdump
    mkdir -p "$log_dir/segment_dump"
    xseg=extract-segments
    command -v extract-segments >/dev/null 2>&1 || xseg="$here/bin/extract-segments"  # no Kaldi on PATH
    $xseg scp,p:$scp $segment ark,scp:${scp_dump_name}.ark,${scp_dump_name}.scp || exit 1
  fi
  split_segments=""
  for n in $(seq $nj); do split_segments="$split_segments $log_dir/segments.$n"; done
  split_list ${scp_dump_name}.scp $split_segments || exit 1
  run_jobs "$log_dir/segments.JOB" "--scp_type=segment"
  for n in $(seq $nj); do cat "$feat_dir/melspec_$name.$n.scp" || exit 1; done > "$data_dir/feats.scp"
  rm "$log_dir"/segments.*
elif [ -f "$scp" ]; then
  split_scp=""
  for n in $(seq $nj); do split_scp="$split_scp $log_dir/wav_${name}.$n.scp"; done
  split_list "$scp" $split_scp || exit 1
  run_jobs "$log_dir/wav_${name}.JOB.scp" ""
  for n in $(seq $nj); do cat "$feat_dir/melspec_$name.$n.scp" || exit 1; done > "$data_dir/feats.scp"
  rm "$log_dir"/wav_${name}.*.scp
else
  echo "$0: Neither scp file nor segment file exists... something is wrong!"
  exit 1
fi

if $write_utt2num_frames; then
  for n in $(seq $nj); do cat "$feat_dir/melspec_$name.$n.len" || exit 1; done > "$data_dir/utt2num_frames"
fi
if $compute_cmvn; then  # JOB partial stats -> one global cmvn.ark (a host sum; no collective needed)
  stats_files=""
  for n in $(seq $nj); do stats_files="$stats_files $feat_dir/cmvn_${name}.$n.mat"; done
  PYTHONPATH="$here${PYTHONPATH:+:$PYTHONPATH}" python3 -c \
    "import sys; from speech_recognition_tools_amd.cmvn import sum_stats_files; sum_stats_files(sys.argv[2:], sys.argv[1])" \
    "$data_dir/cmvn.ark" $stats_files || exit 1
fi
echo "$0: Finished computing FDLP spectrum features for $name"
