"""Phase probe of the fused small-batch Ed25519 kernel (variant library built with
-DCBFT_ED_PHASES=1, selected by $CBFT_LIB): a few key-table batches of 1 and 16 signatures."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "concord-bft_amd"), HERE]
import numpy as np  # noqa: E402
import torch  # noqa: E402  (initialised before the library touches HIP)

torch.cuda.set_device(0)
import cbft_hipcrypto as cb  # noqa: E402
import workload  # noqa: E402

ss = workload.make_sigset(64, nkeys=16, msg_len=256, seed=5)
ctx = cb.Context(device=0)
tid = ctx.load_keys(ss.pk)
for n in (1, 16, 16, 16):
    msgs = [bytes(ss.blob[256 * i: 256 * i + 256]) for i in range(n)]
    bm = ctx.verify(tid, ss.key_idx[:n], ss.sig[:n], msgs)
    print("n", n, "verdicts", np.unpackbits(np.frombuffer(bm, dtype=np.uint8), bitorder="little")[:n].sum(), flush=True)
ctx.close()

# the same batches with their inputs in HBM (cbft_ed25519_verify_fixed_device): the phase times
# without the zero-copy path's PCIe reads

dev = torch.device("cuda", 0)
ctx = cb.Context(device=0)
tid = ctx.load_keys(ss.pk)
d_k = torch.from_numpy(np.ascontiguousarray(ss.key_idx).view(np.int32).copy()).to(dev)
d_sig = torch.from_numpy(np.ascontiguousarray(ss.sig.reshape(-1)).copy()).to(dev)
d_msg = torch.from_numpy(np.ascontiguousarray(ss.blob).copy()).to(dev)
out = torch.zeros(1, dtype=torch.int64, device=dev)
for n in (1, 16, 16):
    ctx.verify_fixed_device(tid, 0, d_k.data_ptr(), d_sig.data_ptr(), d_msg.data_ptr(), 256, n, out.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print("device n", n, "verdict bits", int(out.cpu().item()).bit_count(), flush=True)
ctx.close()
