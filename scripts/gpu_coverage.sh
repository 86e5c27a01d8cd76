#!/usr/bin/env bash
# (1) The N-rank bench path end to end on one GPU: `bench.py --gpus 2` (spawn_ranks, 2 ranks on
#     cuda:0, gloo: PT_BENCH_REHEARSE=1), the default line with its configs[4] leg.
# (2) Which kernels the -m gpu suite launches: the suite under rocprofv3 --kernel-trace; the kernel
#     names go to gpurun_out/$TAG/kernels_launched.txt (tests/test_kernel_coverage.py compares them with
#     the kernels the library's code objects hold).
set -euo pipefail
TAG=${1:-coverage}; OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
PT_BENCH_REHEARSE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 5 > "$OUT/rehearse_c2_n2.json" 2> "$OUT/rehearse.err" || { tail -30 "$OUT/rehearse.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/rehearse_c2_n2.json').read().strip().splitlines()[-1]);print('rehearsal', d['n_gpus'], d['ms_per_step'], d['config']['image'], d['configs4']['verified'], d.get('launch_variant'))"
timeout -k 10 1000 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o suite -- python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/suite.log" 2>&1 || { tail -30 "$OUT/suite.log"; exit 1; }
tail -2 "$OUT/suite.log"
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
names = set()
for f in glob.glob(out + "/prof/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        names.add(row["Kernel_Name"])
open(out + "/kernels_launched.txt", "w").write("\n".join(sorted(names)) + "\n")
print(len(names), "distinct kernels launched")
PY
