set -eo pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for d in 3 1; do
  cd /tmp && rm -rf /tmp/tt$d
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/tt$d -o run -- \
      python3 $R/bench.py --steps 8 --warmup 2 --cpu-budget 0 --side-steps 0 --depth $d > $O/tt_bench_d$d.log 2>&1
  cd $R
  python3 tools/trace_timeline.py /tmp/tt$d > $O/tt_timeline_d$d.txt
  cat $O/tt_timeline_d$d.txt
done
