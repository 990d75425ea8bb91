"""Install the in-tree libbicos_amd.so with the reference's installed layout and build a
downstream C++ project against it (used by __graft_entry__.build() and tests/test_cpp_api.py).

The reference installs include/BICOS/{common,match,config}.hpp next to libBICOS.so
(CMakeLists.txt:82-104); this repository's CMakeLists.txt installs the same names, plus
find_package(BICOS) support. tests/cpp/consumer is a reference-style caller.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def install_and_build_consumer(prefix, bdir, quiet=True):
    """cmake-install the in-tree libbicos_amd.so with the reference's header layout into
    `prefix` (CMakeLists.txt, -DBICOS_PREBUILT_LIB), then configure and build the downstream
    project tests/cpp/consumer (find_package(BICOS) + tests/cpp/ref_style.cpp) in `bdir`."""
    lib = os.path.join(ROOT, "libbicos_amd", "libbicos_amd.so")
    kw = dict(check=True, capture_output=quiet)
    subprocess.run(["cmake", "-S", ROOT, "-B", os.path.join(bdir, "pkg"),
                    "-DBICOS_PREBUILT_LIB=" + lib, "-DCMAKE_INSTALL_PREFIX=" + prefix], **kw)
    subprocess.run(["cmake", "--install", os.path.join(bdir, "pkg")], **kw)
    subprocess.run(["cmake", "-S", os.path.join(ROOT, "tests", "cpp", "consumer"), "-B", bdir,
                    "-DCMAKE_PREFIX_PATH=" + prefix], **kw)
    subprocess.run(["cmake", "--build", bdir], **kw)
    return os.path.join(bdir, "ref_style")
