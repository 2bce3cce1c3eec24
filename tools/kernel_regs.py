"""Register / LDS / spill use of the library's gfx950 kernels (from the code
object's metadata notes).  Usage: python tools/kernel_regs.py [substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.environ.get("OCFFM_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "one-class-ffm_amd", "libocffm.so")


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    for blk in notes.split("  - .agpr_count:")[1:]:
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
        name = get("name")
        if pat not in name:
            continue
        agpr = blk.split()[0]
        print(f"{name[:90]:90s} vgpr {get('vgpr_count'):>4} agpr {agpr:>4} sgpr {get('sgpr_count'):>4} "
              f"spill {get('vgpr_spill_count')} scratch {get('private_segment_fixed_size')} lds {get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
