"""The JNI shim (integration/jni/otsdb_agg_jni.c) and its Java side
(integration/java/net/opentsdb/core) agree with each other and with the
C-ABI header, checked textually (no JDK in this image, so neither is
compiled here).  CPU only."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "integration", "jni", "otsdb_agg_jni.c")
JAVA = os.path.join(ROOT, "integration", "java", "net", "opentsdb", "core",
                    "GpuAggregation.java")
HDR = os.path.join(ROOT, "include", "otsdb_agg.h")


def _read(p):
    with open(p) as f:
        return f.read()


def test_shim_calls_only_declared_entry_points():
    hdr = _read(HDR)
    declared = set(re.findall(r"\b(otsdb_\w+)\s*\(", hdr))
    code = re.sub(r"/\*.*?\*/", "", _read(JNI), flags=re.S)
    calls = set(re.findall(r"\b(otsdb_\w+)\s*\(", code))
    assert calls, "the shim calls the engine"
    assert calls <= declared, calls - declared


def test_java_natives_have_jni_symbols():
    java = _read(JAVA)
    c = _read(JNI)
    natives = re.findall(r"static native \w+ (\w+)\(([^)]*)\)", java, re.S)
    assert len(natives) >= 4
    for name, params in natives:
        n_java = len([p for p in params.split(",") if p.strip()])
        m = re.search(r"Java_net_opentsdb_core_GpuAggregation_%s\(([^)]*)\)"
                      % name, c, re.S)
        assert m, name
        n_c = len([p for p in m.group(1).split(",") if p.strip()])
        assert n_c == n_java + 2, (name, n_c, n_java)  # JNIEnv*, jclass


def test_packed_spec_layout_matches():
    java = _read(JAVA)
    c = _read(JNI)
    jv = dict((k, int(v)) for k, v in
              re.findall(r"(SPEC_\w+) = (\d+)", java))
    body = re.search(r"enum \{\s*(SPEC_[^}]*)\}", c, re.S).group(1)
    names = [x.strip() for x in body.split(",") if x.strip()]
    assert [jv[n] for n in names] == list(range(len(names)))
