"""Dev tool: per-kernel VGPR / spill / LDS usage of the gfx950 code object in
build/igx_device_p*.o (reads the AMDGPU metadata notes).
usage: kernel_resources.py [name filter] [objects...]"""
import glob
import re
import subprocess
import sys

LLVM = "/opt/rocm/llvm/bin"
pat = sys.argv[1] if len(sys.argv) > 1 else "k_"
objs = sys.argv[2:] or sorted(glob.glob("ignis-masterthesis_amd/build/igx_device_p*.o"))
notes = ""
for obj in objs:
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=/tmp/_fat.bin", obj, "/tmp/_host.o"], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=/tmp/_fat.bin",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=/tmp/_dev.co"], check=True)
    notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", "/tmp/_dev.co"], capture_output=True, text=True).stdout
for b in notes.split(".name:")[1:]:
    name = b.split("\n")[0].strip()
    if pat not in name:
        continue
    dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", b) or [None, "-"])[1]
    print(f"{dn[:70]:70s} vgpr {g('vgpr_count'):>4} spill {g('vgpr_spill_count'):>3} priv {g('private_segment_fixed_size'):>4} lds {g('group_segment_fixed_size'):>6}")
