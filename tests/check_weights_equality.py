#!/usr/bin/env python
"""Reference path shim (reference tests/check_weights_equality.py) -> tools/check_weights_equality.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from check_weights_equality import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
