"""Run bench.py with torch.cuda.graph's __exit__ reporting an exception raised
inside the captured block before capture_end runs (a failed capture can crash
there and hide the original error)."""
import os
import runpy
import sys
import traceback

import torch

_orig = torch.cuda.graphs.graph.__exit__


def _exit(self, *exc):
    if exc[0] is not None:
        print("EXCEPTION INSIDE CAPTURE:", file=sys.stderr, flush=True)
        traceback.print_exception(*exc)
        sys.stderr.flush()
    return _orig(self, *exc)


torch.cuda.graphs.graph.__exit__ = _exit
sys.argv = [os.path.join(os.path.dirname(__file__), "..", "..", "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
