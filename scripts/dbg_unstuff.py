import sys, os
sys.path.insert(0, "image-compression_amd"); sys.path.insert(0, ".")
import numpy as np
import icx
from tests.oracle_ffi import load_decode_golden
meta, jpgs, pxs = load_decode_golden()
c = icx.Codec(0)
names = ["c130x250_s2_q95", "rst7_130x250_444", "c66x130_s1_q50"]
res = c.decode_jpg_batch([jpgs[n] for n in names], subsampling=1)
print([r[0] for r in res])
