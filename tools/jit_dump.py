"""Write the generated query header of a shape (sgq_query.h) into a directory and report the
register / scratch usage of the specialised advance kernel (offline hipcc of p2_jit.hip).

    python tools/jit_dump.py [shape|c2] [variant_flags] [outdir]
"""
import importlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sa = importlib.import_module("siddhi-1_amd")
synth = importlib.import_module("siddhi-1_amd.synth")


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/sgjit"
    if name == "c2":
        q = synth.C2_QUERY
    else:
        from test_gpu_parity import SHAPES
        q = SHAPES[name]
    app = sa.parse_app(q)
    cq = sa.compile_query(app, app.queries[0], sa.StringDictionary())
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "sgq_query.h"), "w") as f:
        f.write(sa.jit_check(cq.ir, flags))
    csrc = os.path.join(ROOT, "siddhi-1_amd", "csrc")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
           "--cuda-device-only", "-include", "hip/hip_runtime.h", "-c", "-I", out, "-I", csrc, "-I", os.path.join(ROOT, "include"),
           "-Rpass-analysis=kernel-resource-usage", "-save-temps=obj", "-o", os.path.join(out, "adv.o"),
           os.path.join(csrc, "p2_jit.hip")]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=out)
    for line in r.stderr.splitlines():
        if any(k in line for k in ("Function Name", "VGPRs:", "AGPRs", "ScratchSize", "Occupancy", "SGPRs Spill",
                                    "VGPRs Spill", "LDS Size", "error")):
            print(line.split("remark: ")[-1])
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == "__main__":
    main()
