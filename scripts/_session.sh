source scripts/gpu_steps.sh
rm -f $OUT/status.log
run build 600 python -c "import __graft_entry__ as g; g.build()"
run pytest_gpu 900 python -m pytest tests -m gpu -q
