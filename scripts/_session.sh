source scripts/gpu_steps.sh
rm -f $OUT/status.log
run build 600 python -c "import __graft_entry__ as g; g.build()"
run t_ln 600 python -m pytest tests/test_hip_kernels.py -m gpu -x -q -k "layer_norm"
run gmm 300 python scripts/gmm_probe.py
