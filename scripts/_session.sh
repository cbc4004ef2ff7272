source scripts/gpu_steps.sh
rm -f $OUT/status.log
run build 600 python -c "import __graft_entry__ as g; g.build()"
run t_fuse 600 python -m pytest tests/test_hipfuse.py tests/test_hipgraph.py -m gpu -x -q
run traces 600 python scripts/dump_traces.py $OUT/traces
run bench_graph 900 python bench.py --steps 5 --warmup 3 --hipgraph
run bench_fuse 900 python bench.py --steps 5 --warmup 2 --executors hipex,hipfuse,torch
