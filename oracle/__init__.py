"""oracle/ — TEST INFRASTRUCTURE ONLY.

CPU restatements used as checkers by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Nothing under mandalorion_amd/ imports this package; the product path is the HIP library.

  poa_ref.c    abPOA v1.4.1 restatement (PARITY UNPINNED: abPOA is absent from the container)
  poa.py       ctypes loader for it
  cluster.py   (see module) restatement of the clustering half, pinned by reference fixtures
"""
