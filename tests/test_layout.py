"""CPU: the row-split register layouts of k_step_split (RULE 5 / 6) are the
bijection they claim (tables parsed from the kernel source)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import split_layout  # noqa: E402


def test_split_tables_route_rows():
    src = open(os.path.join(ROOT, "lifeapi_amd", "csrc", "split_layout.hpp")).read()
    assert split_layout.check(src) == [2, 4, 8, 16]
