"""Ed25519 key-table load timing: cbft_ed25519_load_keys of N client keys (default 4,096), median
of 3 load + unload rounds after one warm-up, on the library $CBFT_LIB selects (A/B variants)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "concord-bft_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
pk = workload.pubkeys(workload.key_seeds(n))
ctx = cb.Context(device=0)
ts = []
for r in range(4):
    t = time.perf_counter()
    tid = ctx.load_keys(pk)
    ts.append((time.perf_counter() - t) * 1e3)
    ctx.unload_keys(tid)
ts = sorted(ts[1:])
print(f"{os.environ.get('CBFT_LIB', 'default')}: load {n} keys median {ts[1]:.1f} ms (all {ts})")
ctx.close()
