"""Diagnostics for the fallback Huffman pass (k_flate_tok): scan the structural
fuzz's unmodified flate files with every block forced through it
(RIO_CFG_FLATE_TOK_ONLY) and compare with the oracle. Usage: diag_tok.py [span]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import test_structural_fuzz_gpu as T
    from base_amd.recordio import gpu
    from oracle import oracle
    span = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
    ctx = gpu.Context(0, max_span_bytes=span, flate_tok_only=True)
    bad = 0
    for f in range(3):
        data = T._file(["flate"], 100 * f + 1)
        print("file", f, len(data), flush=True)
        items, err = T._scan(data, ctx)
        ref = oracle.scan(data, read_trailer=False)
        ok = items == ref.items and err == ref.err
        bad += not ok
        print("file", f, "items", len(items), "ref", len(ref.items), "err", repr(err), "ok", ok, flush=True)
    ctx.close()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
