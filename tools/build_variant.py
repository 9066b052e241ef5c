"""Build a compile-time variant of the native library for a same-box A/B: one source (igemm.hip by
default, --src <stem> for another) recompiled with extra -D flags, linked with the other (unchanged)
objects into _native/libpcmp_hip_<name>.so; run it with PCMP_LIB=<that path>.

Usage: python tools/build_variant.py <name> [--src f32] -DPCMP_EPI_COAL=1 -DPCMP_BN_GROUP=1
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp._build as b  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    stem = "igemm"
    if defs[:1] == ["--src"]:
        stem, defs = defs[1], defs[2:]
    b.build(verbose=False)   # the default objects
    inc, libdir, abi = b._torch_paths()
    flags = b._common_flags(inc, abi)
    src = b.CSRC / f"{stem}.hip"
    obj = b.OBJ_DIR / f"{stem}_{name}_hip.o"
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast", *flags, *defs,
                    "-x", "hip", "-c", str(src), "-o", str(obj)], check=True)
    objs = [obj if o.name == f"{stem}_hip.o" else o for o in
            (b.OBJ_DIR / (s.stem + ("_hip.o" if s.suffix == ".hip" else "_cpp.o")) for s in b.sources())]
    lib = b.OUT_DIR / f"libpcmp_hip_{name}.so"
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs),
                    f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                    "-ltorch_hip", "-fopenmp"], check=True)
    print(lib)


if __name__ == "__main__":
    main()
