import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# A/B runs on the GPU box: MMSEQ_BENCH_LIB=ab/libmmseq_<name>.so points the tests at another build
# of the library (tools/ab_build.sh); unset, the in-tree build is loaded as always.
if os.environ.get("MMSEQ_BENCH_LIB"):
    from multimodal_sequencing_amd import _native as _nat
    _nat.LIB_PATH = os.path.join(ROOT, os.environ["MMSEQ_BENCH_LIB"])
