# draw()'s SDMA host-frame path under rocprofv3 (kernel + memory-copy trace): one SDMA setting of tools/copy_ab.py
# (SDMA_SETTINGS, default 3:0 = SDMA, the library's writer), one round.
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
rm -rf $R/gpurun_out/prof_sdma
SETTINGS=${SDMA_SETTINGS:-3:0} ROUNDS=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof_sdma -o run -- python3 $R/tools/copy_ab.py > $R/gpurun_out/prof_sdma.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 $R/gpurun_out/prof_sdma.log; find $R/gpurun_out/prof_sdma -name "*stats*.csv" | head
echo "async-copy errors: $(grep -c 'bad original signal' $R/gpurun_out/prof_sdma.log)"
exit $rc
