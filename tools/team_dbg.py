"""Dev helper: one config-5-shaped -S group through the GPU POA under the current MANDO_TEAM /
MANDO_POA_DBG, compared with the oracle."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mandalorion_amd import poa
from oracle import poa as opoa
from tests import poa_cases
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
g = poa_cases.noisy_groups(n, (8300, 8700), (int(os.environ.get("DEPTH", 20)),) * 2, seed=55)[1]
want = opoa.consensus_batch(g, seeding=[1] * n)
try:
    got = poa.poa_consensus_batch(g, seeding=[1] * n)
    print(os.environ.get("MANDO_TEAM"), os.environ.get("MANDO_POA_DBG"), "equal" if got == want else "DIFFERENT")
except Exception as e:
    print(os.environ.get("MANDO_TEAM"), os.environ.get("MANDO_POA_DBG"), "ERROR", e)
