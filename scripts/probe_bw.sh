# bucket-walk phase timings (SHD_BW_PROBE bits: 1 no sort, 2 no walks, 4 no outcome writes), rocprof per run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for P in ${PROBES:-0 2 7}; do
  SHD_BW_PROBE=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/probe_$P -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/probe_$P.json 2> gpurun_out/probe_$P.err || exit 1
done
