#!/usr/bin/env python3
"""Drop-in `defineIsoforms.py` of this build (same -i -p -c -g -w -m -W -n -j -u -d -a arguments);
clustering on host C++ threads, orientation + POA consensus on the GPU (mandalorion_amd/define.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mandalorion_amd.define import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
