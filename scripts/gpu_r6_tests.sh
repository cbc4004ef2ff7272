#!/bin/bash
# Round-6 GPU checks: the new tests first (symbolic shapes, training trajectory, dQ-from-dS at the 7B
# shape with token-major dO, Gemma-like model), each a bounded step.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run t_sym 400 $PYT tests/test_symbolic_shapes.py -m gpu
run t_traj 400 $PYT tests/test_gpu_7b_shape.py -m gpu -k trajectory
run t_dqds 400 $PYT tests/test_hip_kernels.py -m gpu -k dq_from_ds
run t_models 400 $PYT tests/test_gpu_models.py -m gpu -k "litgpt_fwd_bwd"
