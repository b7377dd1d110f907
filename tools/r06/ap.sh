#!/bin/bash
# round-6 call AP: bf16 ensemble training, separate processes, current build vs the build before the chunked
# BN finalize (libdfd_hip_bnprev.so), interleaved
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/r06; mkdir -p $O
for i in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then LIBV=$R/deepfake-video-detection_amd/libdfd_hip_bnprev.so; else LIBV=; fi
    DFD_HIP_LIB=$LIBV timeout -k 10 300 python bench_temporal.py --model ensemble_train --clips 8 --steps 8 --warmup 2 --no-cpu-baseline --ens-dtypes bf16 > $O/ap_${v}$i.jsonl 2> $O/ap_${v}$i.err || { echo "$v FAILED"; tail -3 $O/ap_${v}$i.err; exit 1; }
    echo "$v run $i: $(python -c "import json;print(json.loads(open('$O/ap_${v}$i.jsonl').readline())['ms_per_step'])") ms"
  done
done
