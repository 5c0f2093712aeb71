# C3 (configs[2]) diagnostics: the per-level trial counters and round timeline (ATZ_TIMING=2), then a
# kernel trace of one step (tools/trace_gaps.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r6c3}; mkdir -p $O
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'.'); from antiz_amd import datagen; datagen.cached('c3','/tmp/atz_bench_cache')" > $O/gen.log 2>&1 || exit 3
ATZ_TIMING=2 timeout -k 10 300 python3 bench.py --workload c3 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/timing.json 2> $O/timing.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o t --output-format csv -- python3 bench.py --workload c3 --steps 1 --warmup 1 --no-cpu --no-recon --no-h2h > $O/tr.json 2> $O/tr.err || exit 5
python3 tools/trace_gaps.py $O/tr > $O/gaps.txt 2>&1 || true
cp $O/tr/*/*kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/tr -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/tr
echo done
