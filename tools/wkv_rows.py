"""WKV per-row cost, cold vs warm: one slot, 64-token prompt through infer (16 heads x 1 segment
WKV workgroups loop over the rows); stamps of layer 5 (RWKVTTS_WKV_STAMPS debug hook)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
path = "/tmp/wkv_rows.bin"
os.environ["RWKVTTS_WKV_STAMPS"] = path
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=4, token_chunk_size=512, use_graphs=False)
for rep in range(3):
    inp = rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(range(20000, 20064)))], 512)
    rt.reset_slot(0)
    rt.infer(inp, head_rows=0, slots=[0])
    st = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)[:16].astype(np.int64)  # 16 heads x 1 seg
    row0 = st[:, 6] - st[:, 0]
    row1 = st[:, 7] - st[:, 6]
    print(f"rep {rep}: row0 (incl. prologue) median {np.median(row0):.0f}  row1 median {np.median(row1):.0f} cycles;"
          f" phases row0: " + " ".join(f"{np.median(st[:, k+1]-st[:, k]):.0f}" for k in range(5)))
