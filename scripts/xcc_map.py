#!/usr/bin/env python3
"""Diagnostics: the XCD (HW_REG_XCC_ID) of each workgroup of a 256-block,
one-workgroup-per-CU grid, checked against the placement group_role assumes
(blocks b and b + 8 share an XCD).  python scripts/xcc_map.py"""
import ctypes
import os
import sys
from collections import Counter

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "seq2seq_abcd-vae_amd"))
from modules import _native as N  # noqa: E402

lib = N.lib()
lib.abcd_debug_xcc_map.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for rep in range(3):
    out = torch.zeros(2 * 256, dtype=torch.int32, device="cuda")
    assert lib.abcd_debug_xcc_map(ctypes.c_void_p(out.data_ptr()), 256, None) == 0
    torch.cuda.synchronize()
    v = out.cpu().view(256, 2)
    xcc = [int(x) & 0xF for x in v[:, 0]]
    raw = Counter(int(x) for x in v[:, 0])
    by_mod = {m: Counter(xcc[b] for b in range(m, 256, 8)) for m in range(8)}
    uniform = all(len(c) == 1 for c in by_mod.values())
    print(f"rep {rep}: raw XCC_ID values {dict(raw)}; per-XCD block count {dict(Counter(xcc))}")
    print(f"   blocks b % 8 = m -> XCC ids: {[dict(c) for c in by_mod.values()]}  (one XCD per residue: {uniform})")
    print(f"   first 16 blocks: xcc {xcc[:16]}  hw_id {[hex(int(h)) for h in v[:16, 1]]}")
