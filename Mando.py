#!/usr/bin/env python3
"""Drop-in `Mando.py` of this build: same CLI as Mandalorion's Mando.py; runs the D module on the GPU
(see mandalorion_amd/mando.py).  Example: python3 Mando.py -p out -f reads.fasta -M D"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mandalorion_amd.mando import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
