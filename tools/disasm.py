"""Disassemble every gfx950 code object of a built library into DIR/<n>.s (diagnostic).
    python tools/disasm.py [lib] [dir]"""
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else "gibbssampling_amd/libgibbs_hip.so"
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/disasm"
os.makedirs(out, exist_ok=True)
subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, f"{out}/fatbin"], check=True)
data = open(f"{out}/fatbin", "rb").read()
st = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
for i, s in enumerate(st):
    e = st[i + 1] if i + 1 < len(st) else len(data)
    open(f"{out}/b{i}", "wb").write(data[s:e])
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={out}/b{i}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}/c{i}.o"], capture_output=True)
    if r.returncode:
        continue
    s_ = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", f"{out}/c{i}.o"], capture_output=True, text=True).stdout
    open(f"{out}/{i}.s", "w").write(s_)
    names = sorted(set(re.findall(r"<(gs_\w+|void gs_\w+)", s_)))[:3]
    print(i, len(s_.splitlines()), names)
