"""CPU tests of the drop-in boundary: the C-ABI library builds, loads and
exports every symbol include/rio_gpu.h declares; host-only entry points work
without a GPU; the host writer restates the reference's layout."""
import ctypes
import os
import re

from conftest import ROOT


def declared_functions():
    with open(os.path.join(ROOT, "include", "rio_gpu.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(rio_[a-z_0-9]+)\s*\(", src))
    return sorted(names)


def test_header_lists_exports():
    from base_amd.recordio import gpu
    assert set(declared_functions()) == set(gpu.EXPORTS)


def test_library_exports_all_symbols(gpu_lib):
    missing = [n for n in declared_functions() if not hasattr(gpu_lib, n)]
    assert missing == []
    assert gpu_lib.rio_abi_version() == 2


def test_build_id_matches_tree(gpu_lib):
    """The loaded library was built from this tree's sources and flags: its
    rio_build_id() is the tree hash (base_amd/build.py), and a library with
    another id is refused."""
    from base_amd import build as B
    from base_amd.recordio import gpu
    assert gpu.build_id() == B.tree_build_id() == B.lib_build_id(B.LIB)
    assert len(gpu.build_id()) == 16
    assert B.tree_build_id(B.FLAGS + ["-DX"]) != B.tree_build_id()


def test_codec_registry_lookup(gpu_lib):
    """registry.go:51-73 + recordioflate/zstd Init: name before the first space."""
    from base_amd.recordio.gpu import RioError

    def look(vals):
        arr = (ctypes.c_char_p * max(len(vals), 1))(*[v.encode() for v in vals])
        codec = ctypes.c_int32(-1)
        err = RioError()
        rc = gpu_lib.rio_codec_for_transformers(arr, len(vals), ctypes.byref(codec), ctypes.byref(err))
        return rc, codec.value, err.msg.decode()

    assert look([]) == (0, 0, "")
    assert look(["flate"])[:2] == (0, 1)
    assert look(["flate 5"])[:2] == (0, 1)
    assert look(["zstd -1"])[:2] == (0, 2)
    # not decoded here -> RIO_ERR_FALLBACK (23): the shim's recordio.NewShardScanner
    # decodes it, or reports the reference's own "not found" text
    rc, _, msg = look(["nonexistent 3"])
    assert rc == 23 and msg == "Transformer nonexistent 3 not found"
    rc, _, msg = look(["flatex"])
    assert rc == 23 and msg == "Transformer flatex not found"
    # a chain: reverse-order untransform (registry.go:121-146), up to 4 stages
    assert look(["flate", "zstd"])[:2] == (0, 0x10000 | (2 << 8) | 1 | (2 << 2))
    assert look(["zstd 3", "flate", "flate 9"])[:2] == (0, 0x10000 | (3 << 8) | 2 | (1 << 2) | (1 << 4))
    assert look(["flate"] * 5)[0] == 23  # longer: the reference scanner
    assert look(["flate", "snappy"])[0] == 23


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors agree with the C compiler's layout of include/rio_gpu.h."""
    from base_amd.recordio import gpu
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rio_gpu.h"\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(rio_error), sizeof(rio_config),'
                   ' sizeof(rio_batch), offsetof(rio_batch, err), offsetof(rio_batch, kernel_ms),'
                   ' sizeof(rio_reader)); return 0;}\n')
    exe = tmp_path / "sz"
    import subprocess
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(gpu.RioError), ctypes.sizeof(gpu.RioConfig), ctypes.sizeof(gpu.RioBatch),
            gpu.RioBatch.err.offset, gpu.RioBatch.kernel_ms.offset, ctypes.sizeof(gpu.RioReader)]
    assert got == want


def test_writer_layout_known_answers():
    from base_amd.recordio import format as F
    from base_amd.recordio.writer import write_file, WriterOpts
    assert len(write_file([])) == 32768
    assert len(write_file([], trailer=b"x")) == 65536
    d = write_file([b"a" * 32740], WriterOpts(MaxItems=1))
    # header chunk + a 32744-byte block (4-byte varint header; 2 chunks)
    assert len(d) == 3 * 32768
    # chunk header fields (chunk.go:31-53)
    magic, crc, flag, size, total, index = __import__("struct").unpack_from("<8sIIIII", d, 32768)
    assert magic == F.MAGIC_PACKED and flag == 0 and size == 32740 and total == 2 and index == 0
    import zlib
    assert crc == zlib.crc32(d[32768 + 12:32768 + 28 + size])
    # padding is deadbeef (chunk.go:77-82)
    tail = d[2 * 32768 + 28 + 4: 2 * 32768 + 28 + 4 + 8]
    assert tail == bytes.fromhex("deadbeefdeadbeef")


def test_uvarint_go113_semantics():
    from base_amd.recordio.format import uvarint, put_uvarint
    for v in [0, 1, 127, 128, 300, 2 ** 63, 2 ** 64 - 1]:
        assert uvarint(put_uvarint(v)) == (v, len(put_uvarint(v)))
    assert uvarint(b"") == (0, 0)
    assert uvarint(b"\x80\x80") == (0, 0)
    assert uvarint(b"\xff" * 9 + b"\x02") == (0, -10)
    assert uvarint(b"\xff" * 10 + b"\x01") == (0, -11)  # Go 1.13 scans past 10 bytes
