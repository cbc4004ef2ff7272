source scripts/gpu_steps.sh
rm -f $OUT/status.log
run build 600 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py --steps 10 --warmup 3
