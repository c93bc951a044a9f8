import os, sys, subprocess
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import poa_cases
from mandalorion_amd import poa
from oracle import poa as opoa
gs = poa_cases.edge_groups()
want = opoa.consensus_batch(gs)
got = poa.poa_consensus_batch(gs)
print(os.environ.get("MANDO_POA_DBG", "0"), [i for i, (a, b) in enumerate(zip(got, want)) if a != b])
