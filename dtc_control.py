#!/usr/bin/env python3
"""Drop-in CLI for autocorr-delta-a-single-qiskit-fast-controlled-g.py and
-g-optimization.py (``--script``) on the MI355X engine.  See <package>/control_cli.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from __graft_entry__ import load_package  # noqa: E402

if __name__ == "__main__":
    raise SystemExit(load_package().control_cli.main())
