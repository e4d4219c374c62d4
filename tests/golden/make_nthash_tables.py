"""Extract ntHash's constant tables from the reference's prebuilt binary as DATA.

The reference (Codfishz/Sketch-for-RNA-seq) does not vendor ntHash; it links bcgsc ntHash >= 2.3
(`build.sh:34`, `src/sketch.cpp:7`). Its checked-in `build/test` (Mach-O arm64) statically embeds
ntHash's lookup tables. This script only READS bytes at the table offsets recorded in SURVEY.md
§8c (file offset = vmaddr - 0x100000000); the binary is never executed or loaded.

Output: tests/golden/nthash_tables.json (committed). Run in the dev container only:
    python tests/golden/make_nthash_tables.py
"""
import hashlib
import json
import os
import struct
import sys

SRC = "/root/reference/build/test"
BASE = 0x100000000
# name -> (vmaddr, count, element size)
TABLES = {
    "SEED_TAB": (0x100039F00, 256, 8),
    "CONVERT_TAB": (0x100039280, 256, 1),
    "RC_CONVERT_TAB": (0x100039E00, 256, 1),
    "DIMER_TAB": (0x100039D80, 16, 8),
    "TRIMER_TAB": (0x100039B80, 64, 8),
    "TETRAMER_TAB": (0x100039380, 256, 8),
    "A31L": (0x10003A9E8, 31, 8), "C31L": (0x10003AAE0, 31, 8),
    "G31L": (0x10003A8F0, 31, 8), "T31L": (0x10003A7F8, 31, 8), "N31L": (0x10003A700, 31, 8),
    "A33R": (0x10003AEF0, 33, 8), "C33R": (0x10003AFF8, 33, 8),
    "G33R": (0x10003ADE8, 33, 8), "T33R": (0x10003ACE0, 33, 8), "N33R": (0x10003ABD8, 33, 8),
}


def main(out_path):
    blob = open(SRC, "rb").read()
    out = {"source": "reference build/test (data bytes only)",
           "source_sha256": hashlib.sha256(blob).hexdigest(), "tables": {}}
    for name, (addr, n, sz) in TABLES.items():
        off = addr - BASE
        raw = blob[off:off + n * sz]
        vals = list(struct.unpack("<%d%s" % (n, "Q" if sz == 8 else "B"), raw))
        out["tables"][name] = [("0x%016x" % v) if sz == 8 else v for v in vals]
    with open(out_path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", out_path)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "nthash_tables.json"))
