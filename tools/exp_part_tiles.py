"""Experiment: bench.py with turtle_kv_amd.dist.ROUTED_PART_TILES overridden (the tiles per
routed part of a hash-range build; the library's range builds take any part size).
Usage: python tools/exp_part_tiles.py TILES bench-args..."""
import runpy
import sys

sys.path.insert(0, ".")
import turtle_kv_amd.dist as dist  # noqa: E402

dist.ROUTED_PART_TILES = int(sys.argv[1])
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
