set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/pmcwg
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmcwg/$c -o p --output-format csv -- python3 $R/tools/layer_bench.py --math 2 --only "g_a.2 conv wgrad,g_s.4 tconv wgrad" --reps 5 > $R/gpurun_out/pmcwg/$c.log 2>&1 || exit 1
done
echo DONE
