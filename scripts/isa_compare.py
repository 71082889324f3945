"""Compare the device code of two `hipcc --cuda-device-only -S` outputs kernel by kernel.

A source change meant to leave the shipped kernels untouched (pruning an unused variant, a comment)
is checked here without a GPU: every kernel's instruction stream, labels and comments stripped,
must be identical.  Usage: python scripts/isa_compare.py before.s after.s"""
import re
import sys


def kernels(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r'^(_Z\w+):[^\n]*\n(.*?)s_endpgm', txt, re.M | re.S):
        body = re.sub(r';[^\n]*', '', m.group(2))
        body = re.sub(r'\.L\w+', 'L', body)
        out[m.group(1)] = body
    return out


if __name__ == "__main__":
    b, a = kernels(sys.argv[1]), kernels(sys.argv[2])
    changed = sorted(k for k in b if k in a and b[k] != a[k])
    print(f"kernels: {len(b)} before, {len(a)} after; changed {len(changed)}")
    for k in changed:
        print("  changed:", k)
    for k in sorted(set(b) - set(a)):
        print("  removed:", k)
    for k in sorted(set(a) - set(b)):
        print("  new:", k)
    sys.exit(1 if changed else 0)
