import os, sys, random
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "tests"))
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "sketch-for-rna-seq_amd"))
import numpy as np
import torch
import orc, skq
from skq import synth
os.environ["SKQ_CHAIN"] = "1"; os.environ["SKQ_PROBE"] = "wide"
tx = synth.transcriptome(200, seed=11)
seqs = [tx.seq(t) for t in range(tx.ntx)]
buf, offs = skq.pack_reads(seqs)
for chained in (False, True):
    index = skq.Index([31], len(seqs), skq.build_tables(buf, offs, [31]), seqs=(buf, offs) if chained else None)
    bases, _, _ = synth.reads(tx, 300, 100, seed=12)
    reads = [bases[i*100:(i+1)*100].tobytes() for i in range(300)]
    rb, ro = skq.pack_reads(reads)
    s = skq.Session(index, 300, 100)
    d = skq.DeviceBuffer.from_numpy(rb)
    s.map(d.ptr, None, 300, 100, fixed_len=100)
    s.check()
    out = s.export()
    ref = orc.Index([31], seqs=seqs).map_batch(reads)
    ho = out["hash_offs"]; bad = 0
    for r in range(300):
        got = list(out["hashes"][ho[r]:ho[r+1]]); exp = list(ref["hashes"][r, 0, :ref["hash_cnt"][r, 0]])
        if got != exp:
            bad += 1
            if bad <= 4: print("chained", chained, "read", r, "got", got, "exp", exp, "status", out["status"][r])
    print("chained", chained, "hash mismatches", bad, "of 300")
    s.free(); index.free()
