import sys, runpy
import torch  # noqa: F401  (torch's HIP runtime first)
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
