"""Run bench.py against the package copy in ./ab_old (a previous build kept for same-box A/B runs)."""
import runpy
import sys

sys.path.insert(0, "ab_old")
import aios_amd  # noqa: E402

assert "ab_old" in aios_amd.__file__, aios_amd.__file__
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
