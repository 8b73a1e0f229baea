#!/usr/bin/env python3
"""FETCH_SIZE calibration (see fetch_calib.hip).  Two modes:
  python tools/calib/fetch_calib.py run          one dispatch of each shape (run it under rocprofv3)
  python tools/calib/fetch_calib.py report DIR   bytes read / (FETCH_SIZE KiB * 1024) per shape from
                                                 DIR/run_counter_collection.csv
usage on the GPU box: rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/X -o run --output-format csv \\
  -- python3 tools/calib/fetch_calib.py run  &&  python3 tools/calib/fetch_calib.py report gpurun_out/X"""
import csv
import ctypes
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
BYTES = 1 << 30          # 1 GiB per shape: 4x the Infinity Cache
NAMES = {"stream4": "4 B/lane coalesced", "stream16": "16 B/lane coalesced",
         "hulls4": "GJK tier-0 hull loads (4-lane groups, 32-vertex fp32 SoA hulls, permuted)"}


def run():
    import torch
    lib = ctypes.CDLL(os.path.join(HERE, "build", "libfetch_calib.so"))
    lib.fetch_calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    buf = torch.ones(BYTES // 4, dtype=torch.float32, device=dev)
    nh = BYTES // 384
    perm = torch.randperm(nh, device=dev).to(torch.int32)
    out = torch.zeros(1 << 16, dtype=torch.float32, device=dev)
    flush = torch.empty(BYTES // 4, dtype=torch.float32, device=dev)
    for shape in (0, 1, 2):
        flush.fill_(0.0)                       # evict the Infinity Cache between shapes
        torch.cuda.synchronize()
        assert lib.fetch_calib_run(shape, buf.data_ptr(), nh * 384 if shape == 2 else BYTES, perm.data_ptr(),
                                   out.data_ptr(), 4096) == 0
    print("ok")


def report(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    res = {}
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        if k in NAMES and r["Counter_Name"] == "FETCH_SIZE":
            res[k] = res.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for k, kib in res.items():
        nbytes = (BYTES // 384) * 384 if k == "hulls4" else BYTES
        out[k] = {"shape": NAMES[k], "bytes_read": nbytes, "fetch_size_bytes": kib * 1024,
                  "bytes_per_fetch_byte": round(nbytes / (kib * 1024), 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        report(sys.argv[2])
