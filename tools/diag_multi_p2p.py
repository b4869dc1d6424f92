"""DIAG: does a scatter deliver every byte?  Whole-span ncclSend vs pieces (XSKNF_MULTI_P2P_PIECE)."""
import os, sys, json, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from xsknf_amd import frames, multi
from xsknf_amd.shard import rebase_descs
n = int(sys.argv[1])
dev = torch.device("cuda:0")
b = frames.aligned_batch(n, "imix", seed=frames.SEED)
umem = torch.from_numpy(b.umem).to(dev)
torch.cuda.synchronize()
with multi.MultiDevice([0]) as m:
    secs = m.scatter(0, umem.data_ptr(), umem.numel(), b.descs)
    info = m.shard_info(0)
    su, sv, sd = m.fetch(0, descs=True)
b0, b1 = info["span_lo"], info["span_hi"]
src = b.umem[b0:b1]
bad = np.nonzero(su != src)[0]
want_d = rebase_descs(b.descs, b0, b.umem.size)
dbad = np.nonzero(sd.view(np.uint8).reshape(-1, 16) != want_d.view(np.uint8).reshape(-1, 16))[0]
print(json.dumps({"n": n, "piece": os.environ.get("XSKNF_MULTI_P2P_PIECE"), "span": b1 - b0, "secs": secs,
                  "bad_bytes": int(bad.size), "first_bad": int(bad[0]) if bad.size else None,
                  "last_bad": int(bad[-1]) if bad.size else None, "bad_desc_rows": int(np.unique(dbad).size)}), flush=True)
