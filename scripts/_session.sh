source scripts/gpu_steps.sh
rm -f $OUT/status.log
run build 600 python -c "import __graft_entry__ as g; g.build()"
run t_fuse 600 python -m pytest tests/test_hipfuse.py tests/test_gpu_models.py -m gpu -x -q
run bench_fuse 900 python bench.py --steps 10 --warmup 3 --executors hipex,hipfuse,torch
run bench 900 python bench.py --steps 10 --warmup 3
run traces 600 python scripts/dump_traces.py $OUT/traces_fuse hipex,hipfuse,torch
