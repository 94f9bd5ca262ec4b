"""Per-kernel register / scratch use of the gfx950 code object inside librr.so.

Reads the AMDGPU code-object metadata (llvm-objcopy the .hip_fatbin section,
clang-offload-bundler the gfx950 object out of it, llvm-readelf --notes) and
prints one line per kernel: VGPRs, AGPRs, VGPR spills, scratch bytes, LDS,
demangled name.  `--check` exits 1 if any kernel uses scratch (private segment) memory
(tests/test_kernel_resources.py runs it on every build).

usage: python tools/kernel_resources.py [--check] [--grep SUBSTR] [path/to/librr.so]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _notes(lib):
    """llvm-readelf --notes of every gfx950 code object in the library (one
    offload bundle per translation unit, concatenated in .hip_fatbin)."""
    text = []
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(td, "x.so")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, a in enumerate(starts):
            b = starts[i + 1] if i + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{i}.bin"), os.path.join(td, f"co{i}.o")
            with open(part, "wb") as f:
                f.write(data[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={part}",
                            f"--output={co}", "--unbundle"], check=True, capture_output=True)
            text.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                       text=True).stdout)
    return "\n".join(text)


def kernels(lib):
    notes = _notes(lib)
    out, cur = [], {}
    keys = {".name": str, ".vgpr_count": int, ".agpr_count": int, ".vgpr_spill_count": int,
            ".sgpr_spill_count": int, ".private_segment_fixed_size": int, ".group_segment_fixed_size": int}
    for line in notes.splitlines():
        m = re.match(r"\s*(-\s+)?(\.[a-z_]+):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) and cur:  # a new list item: the previous kernel is complete
            out.append(cur)
            cur = {}
        k = m.group(2)
        if k in keys:
            cur[k] = keys[k](m.group(3))
    if cur:
        out.append(cur)
    return [k for k in out if ".name" in k and ".vgpr_count" in k]


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def main(argv):
    check = "--check" in argv
    grep = None
    if "--grep" in argv:
        grep = argv[argv.index("--grep") + 1]
    paths = [a for a in argv if a.endswith(".so")]
    lib = paths[0] if paths else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "research_image_retrieval_amd", "librr.so")
    ks = kernels(lib)
    names = demangle([k[".name"] for k in ks])
    bad = 0
    for k, n in zip(ks, names):
        # spills into AGPRs (vgpr_spill_count without scratch) cost moves, not
        # memory; scratch is the failure
        spill = k.get(".vgpr_spill_count", 0) + k.get(".sgpr_spill_count", 0)
        scratch = k.get(".private_segment_fixed_size", 0)
        if scratch:
            bad += 1
        if grep is None or grep in n:
            print(f"vgpr {k['.vgpr_count']:3d} agpr {k.get('.agpr_count', 0):3d} spill {spill:3d} "
                  f"scratch {scratch:5d} lds {k.get('.group_segment_fixed_size', 0):6d}  {n[:160]}")
    print(f"{len(ks)} kernels, {bad} using scratch", file=sys.stderr)
    return 1 if (check and bad) else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
