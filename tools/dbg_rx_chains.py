"""Debug helper (GPU): rerun test_gpu_fuzz.test_fuzz_rx_chains' data for one trial and dump the
datagrams whose kernel outputs differ from the oracle (gpurun_out/dbg_rx_chains.json)."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from picotcp_amd import batch  # noqa: E402
from tests.golden import make_ref_rx as M  # noqa: E402

trial = int(sys.argv[1]) if len(sys.argv) > 1 else 1
rng = np.random.default_rng(9100 + trial)
res = []
for gen, fam in ((M.gen_v4, 4), (M.gen_v6, 6)):
    items = gen(rng, 3000)
    buf, off, av = M.pack(items, rng)
    desc = batch.make_desc(off, av)
    d = batch.desc_to_device(desc, "cuda:0")
    if fam == 4:
        wn, wl, wv = O.batch_ipv4(buf, desc)
        net, l4, v = batch.ipv4_checksum_batch(torch.from_numpy(buf).cuda(), d, len(items))
    else:
        wl, wv = O.batch_ipv6(buf, desc)
        l4, v = batch.ipv6_checksum_batch(torch.from_numpy(buf).cuda(), d, len(items))
    torch.cuda.synchronize()
    gl, gv = l4.cpu().numpy().view(np.uint16), v.cpu().numpy()
    for i in np.flatnonzero((gl != wl) | (gv != wv)):
        o, a = int(off[i]), int(av[i])
        k = O.ipv6_walk(buf[o:o + a]) if fam == 6 else None
        res.append(dict(fam=fam, i=int(i), off=o, avail=a, gpu_l4=int(gl[i]), want_l4=int(wl[i]), gpu_v=int(gv[i]),
                        want_v=int(wv[i]), walk=k, hex=bytes(buf[o:o + a]).hex()))
json.dump(res, open("gpurun_out/dbg_rx_chains.json", "w"), indent=1)
print(len(res), "mismatches")
