cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/actp
timeout -k 10 60 ./scripts/bin/mlp_probe x6 rows > gpurun_out/actp/base.log 2>&1 && timeout -k 10 60 ./scripts/bin/mlp_probe_noact x6 rows > gpurun_out/actp/noact.log 2>&1 && tail -2 gpurun_out/actp/base.log && tail -2 gpurun_out/actp/noact.log
