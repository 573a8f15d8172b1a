#!/usr/bin/env python3
"""Drop-in CLI for autocorr-delta-a-single-qiskit-fast-energy*.py (same flags,
same CSV output) on the MI355X engine.  See <package>/energy_cli.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from __graft_entry__ import load_package  # noqa: E402

if __name__ == "__main__":
    raise SystemExit(load_package().energy_cli.main())
