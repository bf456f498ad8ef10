"""SHA-256 of every kernel's machine code in the library (or two libraries
compared).

usage: python scripts/kernel_hashes.py [LIB]            -> JSON {symbol: sha256}
       python scripts/kernel_hashes.py OLD.json LIB     -> per-kernel same / DIFFERENT

Used to show that a source change (e.g. retiring A/B macros from the kernel
sources) left every shipped kernel's code as it was."""
import json
import os
import struct
import sys
import hashlib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from syncfast_amd._lib import _code_objects, LIB_PATH  # noqa: E402


def hashes(path):
    out = {}
    for _, co in _code_objects(path):
        if co[:4] != b"\x7fELF":
            continue
        shoff, = struct.unpack_from("<Q", co, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", co, 0x3A)
        secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + i * shentsize) for i in range(shnum)]
        stro = secs[shstrndx][4]
        names = [co[stro + s[0]: co.index(b"\0", stro + s[0])] for s in secs]
        if b".symtab" not in names:
            continue
        symtab = secs[names.index(b".symtab")]
        strtab = secs[symtab[6]]
        for i in range(symtab[5] // 24):
            st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, symtab[4] + 24 * i)
            nm = co[strtab[4] + st_name: co.index(b"\0", strtab[4] + st_name)].decode()
            if (st_info & 0xF) == 2 and st_size and not nm.endswith(".kd"):  # STT_FUNC
                sec = secs[st_shndx]
                start = sec[4] + (st_value - sec[3])
                out[nm] = hashlib.sha256(co[start: start + st_size]).hexdigest()
    return out


def main():
    if len(sys.argv) == 3:
        old = json.load(open(sys.argv[1]))
        new = hashes(sys.argv[2])
        ok = True
        for k in sorted(set(old) | set(new)):
            st = "same" if old.get(k) == new.get(k) else ("REMOVED" if k not in new else
                                                        "ADDED" if k not in old else "DIFFERENT")
            ok &= st == "same"
            print(f"{st:9s} {k}")
        sys.exit(0 if ok else 1)
    print(json.dumps(hashes(sys.argv[1] if len(sys.argv) > 1 else LIB_PATH), indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
