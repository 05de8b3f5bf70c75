"""Pack the reference fixture (/root/reference/data, read with our own t7 decoder) into
data_cache/fixture/<split>.dgpack.npz so real-data runs work where the reference tree is
not mounted (e.g. the GPU box).  Derived data only; nothing from the reference executes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.data.dataset import PackedDataset, load_index  # noqa: E402

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/data"
DST = sys.argv[2] if len(sys.argv) > 2 else "data_cache/fixture"
os.makedirs(DST, exist_ok=True)
for split in ("train", "validation", "test"):
    pk = PackedDataset.from_index(load_index(SRC, split, build_missing=False))
    out = os.path.join(DST, f"{split}.dgpack.npz")
    pk.save(out)
    print(split, len(pk), pk.num_games, out)
