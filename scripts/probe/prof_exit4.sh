# rocprofv3 on a trivial cooperative launch (exit-time SIGSEGV attribution)
R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pe4 -o run -- $R/scripts/probe/coop > $R/gpurun_out/pe4.log 2>&1; echo rc=$? >> $R/gpurun_out/pe4.log
