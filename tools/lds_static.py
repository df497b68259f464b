"""Static LDS (group_segment_fixed_size) of every kernel in a built library, read from
its gfx950 code objects: the .hip_fatbin section holds one offload bundle a
translation unit; each is unbundled and its AMDGPU metadata note read.

    python tools/lds_static.py [gibbssampling_amd/libgibbs_hip.so]

The live and long sweep kernels address their LDS from 0 (their tables sit at fixed
offsets of the dynamic allocation) and treat a nonzero base as a table fault that sends
every target to the exact rescan: a static __shared__ variable anywhere in them (e.g.
one __syncthreads_or brings) silently turns their fast path off.
tests/test_build_lds.py holds them to 0."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def static_lds(lib):
    """{mangled kernel name: group_segment_fixed_size} over every bundle of lib."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            bpath, cpath = os.path.join(d, f"b{i}"), os.path.join(d, f"c{i}.o")
            open(bpath, "wb").write(data[s:e].rstrip(b"\0") if i + 1 == len(starts) else data[s:e])
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={bpath}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={cpath}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.getsize(cpath):
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", cpath], capture_output=True,
                                   text=True, check=True).stdout
            size = None
            for line in notes.splitlines():
                line = line.strip()
                if line.startswith(".group_segment_fixed_size:"):
                    size = int(line.split(":")[1])
                elif line.startswith(".name:") and size is not None:
                    out[line.split(":", 1)[1].strip()] = size
                    size = None
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "gibbssampling_amd/libgibbs_hip.so"
    for name, size in sorted(static_lds(lib).items()):
        print(size, name)
