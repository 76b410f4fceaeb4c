"""Build an A/B variant of libgnca.so with extra compile flags (measurement builds only).

  python tools/build_variant.py build_ab/lib_x.so -DGNCA_K1_SPLIT_NT=768 ...
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

out, flags = sys.argv[1], sys.argv[2:]
os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
objdir = os.path.join(ROOT, "build", "obj_" + os.path.basename(out).replace(".so", ""))
os.makedirs(objdir, exist_ok=True)
procs, objs = [], []
for src in G.SRCS:
    obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
    objs.append(obj)
    cmd = [G.HIPCC, f"--offload-arch={G.ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-Wno-unused-result",
           *G.SRC_FLAGS.get(os.path.basename(src), []), *flags, f"-I{os.path.join(ROOT, 'include')}", src, "-o", obj]
    procs.append(subprocess.Popen(cmd))
for p in procs:
    if p.wait() != 0:
        sys.exit("hipcc failed")
subprocess.run([G.HIPCC, f"--offload-arch={G.ARCH}", "-shared", "-fPIC", *objs, "-o", out], check=True)
print("built", out, flags)
