S="python -u tools/solve_time.py --reps 20 --shapes 1x400x128,2x400x128 --knobs adaln_cfg=0 adaln_cfg=1 adaln_cfg=2 adaln_cfg=4 adaln_cfg=3 adaln_cfg=5 adaln_cfg=0 adaln_cfg=1 adaln_cfg=5"
bash tools/gpu_steps.sh r06af ab 400 "$S" \
 prof 300 "cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/r06af/prof -o run -- python3 \$GRAFT_REPO_ROOT/tools/solve_time.py --reps 3 --shapes 1x400x128 --knobs adaln_cfg=0 adaln_cfg=1 adaln_cfg=2 adaln_cfg=4"
