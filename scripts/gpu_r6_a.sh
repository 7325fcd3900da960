# round 6, call a: fresh baseline at HEAD — smoke, bench line, step breakdown, PMC bytes per kernel
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a/smoke.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --acc-steps 0 > gpurun_out/r6a/bench.json 2> gpurun_out/r6a/bench.err
bash scripts/prof_step.sh r6a_r50 > /dev/null
mv gpurun_out/r6a_r50_* gpurun_out/r6a/
mkdir -p gpurun_out/pmcstep
i=0
for P in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d /tmp/pmcs$i -o run --output-format csv -- python bench.py --steps 2 --warmup 3 --acc-steps 0 > gpurun_out/r6a/pmc_pass$i.log 2>&1
  f=$(find /tmp/pmcs$i -name '*counter_collection.csv' | head -1)
  python scripts/pmc_summary.py "$f" --last-step --dispatches k_bn_ > gpurun_out/r6a/pmc_pass$i.txt
done
