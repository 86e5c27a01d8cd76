set -euo pipefail
export TMPDIR=/tmp PT_QP_K=30
mkdir -p gpurun_out/v4b4k
for r in 1 2; do
  for v in "X=0" "PT_MI355_BACK=0"; do
    env $v timeout -k 10 120 python3 scripts/v4_perf.py 3840 2160 8 8 | sed "s/^/$v /" >> gpurun_out/v4b4k/ab.txt
    env $v timeout -k 10 120 python3 scripts/v4_perf.py 1920 1080 16 8 | sed "s/^/$v /" >> gpurun_out/v4b4k/ab.txt
  done
done
cut -c1-120 gpurun_out/v4b4k/ab.txt
