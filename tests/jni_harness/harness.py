"""ctypes driver of jni/gdist_jni.c compiled against the test-only JNI
stand-in (tests/jni_harness/jni.h + fake_jvm.c): the natives are called as a
JVM would call them, with fake Java arrays, strings and a pending exception.

build(out) compiles the shim with gcc (-Wall -Wextra -Werror) and links it
to the in-tree libgdist.so; __graft_entry__.build() builds it in-tree
(tests/jni_harness/build/libgdist_jni_test.so) for the GPU test.
"""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
LIBDIR = os.path.join(ROOT, "genome.distance_amd", "gdist")
BUILT = os.path.join(HERE, "build", "libgdist_jni_test.so")
BYTE, INT, LONG, DOUBLE, OBJECT = 1, 2, 3, 4, 5
PREFIX = "Java_org_theseed_genome_distance_gpu_GpuKmerSets_"


def build(out: str = BUILT) -> str:
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["gcc", "-O1", "-fPIC", "-shared", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                    "-I", HERE, "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "jni", "gdist_jni.c"), os.path.join(HERE, "fake_jvm.c"),
                    "-L", LIBDIR, "-lgdist", f"-Wl,-rpath,{LIBDIR}", "-o", out],
                   check=True, capture_output=True, text=True)
    return out


def current():
    """The in-tree build when it is newer than the shim, the stand-ins and libgdist.so, else None."""
    if not os.path.exists(BUILT):
        return None
    srcs = [os.path.join(ROOT, "jni", "gdist_jni.c"), os.path.join(HERE, "fake_jvm.c"), os.path.join(HERE, "jni.h"),
            os.path.join(ROOT, "include", "gdist.h"), os.path.join(LIBDIR, "libgdist.so")]
    t = os.path.getmtime(BUILT)
    return BUILT if all(os.path.getmtime(p) <= t for p in srcs if os.path.exists(p)) else None


class FakeJVM:
    """The shim's natives over fake Java objects."""

    def __init__(self, path: str):
        self.lib = C.CDLL(path)
        L = self.lib
        L.fj_env.restype = C.c_void_p
        L.fj_array.restype = C.c_void_p
        L.fj_array.argtypes = [C.c_int, C.c_int32, C.c_void_p]
        L.fj_data.restype = C.c_void_p
        L.fj_data.argtypes = [C.c_void_p]
        L.fj_string.restype = C.c_void_p
        L.fj_string.argtypes = [C.c_char_p]
        L.fj_set_element.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.fj_exception_class.restype = C.c_char_p
        L.fj_exception_message.restype = C.c_char_p
        L.fj_local_refs.restype = C.c_long
        self.env = L.fj_env()

    # fake Java objects
    def array(self, kind, values):
        ct = {BYTE: C.c_int8, INT: C.c_int32, LONG: C.c_int64, DOUBLE: C.c_double}[kind]
        buf = (ct * max(1, len(values)))(*values)
        return self.lib.fj_array(kind, len(values), buf)

    def zeros(self, kind, n):
        return self.lib.fj_array(kind, n, None)

    def read(self, obj, kind, n):
        ct = {INT: C.c_int32, LONG: C.c_int64, DOUBLE: C.c_double}[kind]
        return list((ct * n).from_address(self.lib.fj_data(obj)))

    def byte_arrays(self, seqs):
        arr = self.lib.fj_array(OBJECT, len(seqs), None)
        for i, s in enumerate(seqs):
            b = self.lib.fj_array(BYTE, len(s), C.c_char_p(s))
            self.lib.fj_set_element(arr, i, b)
        return arr

    def string(self, s):
        return self.lib.fj_string(s.encode())

    def exception(self):
        """(class, message) of the pending exception, cleared; None if none"""
        if not self.lib.fj_pending():
            return None
        e = (self.lib.fj_exception_class().decode(), self.lib.fj_exception_message().decode())
        self.lib.fj_clear()
        return e

    # natives (a JNIEnv*, a jclass, then the Java arguments)
    def call(self, name, restype, *args):
        f = getattr(self.lib, PREFIX + name)
        f.restype = restype
        conv = []
        for a in args:
            if isinstance(a, float):
                conv.append(C.c_double(a))
            elif isinstance(a, int):
                conv.append(C.c_int64(a))
            else:
                conv.append(a)
        return f(C.c_void_p(self.env), None, *conv)

    def call_i(self, name, restype, argtypes, *args):
        """A native whose Java arguments include ints (jint: 32-bit)."""
        f = getattr(self.lib, PREFIX + name)
        f.restype = restype
        f.argtypes = [C.c_void_p, C.c_void_p] + argtypes
        return f(self.env, None, *args)
