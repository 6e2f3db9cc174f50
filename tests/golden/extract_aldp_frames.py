"""Extract the first 512 frames of the reference's ALDP data fixture into tests/golden/aldp_frames.npy.

Source: ecnf/targets/data/aldp_500K_train_mini.h5 (`coordinates` float32[2000, 22, 3], nm), read the way
ecnf/targets/data.py:125-154 (load_aldp) does.  Needs h5py (run with /opt/conda/bin/python3.9 in the dev
container); the output is plain data, so the tests never need h5py or the reference tree.
"""
import os
import sys

import h5py
import numpy as np

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/ecnf/targets/data/aldp_500K_train_mini.h5"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "aldp_frames.npy")

with h5py.File(SRC, "r") as f:
    x = np.asarray(f["coordinates"][:512], dtype=np.float32)
np.save(OUT, x)
print(OUT, x.shape, x.dtype)
