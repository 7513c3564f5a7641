"""The JNI shim (jni/skml_jni.c) type-checks against include/skml.h, and every native the Java
classes declare has its C function (no JDK in this image: jni/test/jni.h is a declaration-only
stand-in used for this check alone; the real build is jni/Makefile with $JAVA_HOME)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shim_compiles_against_the_c_abi():
    out = subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only",
                          "-I", os.path.join(ROOT, "jni", "test"), "-I", os.path.join(ROOT, "include"),
                          os.path.join(ROOT, "jni", "skml_jni.c")], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


def test_every_java_native_has_a_c_function():
    java = open(os.path.join(ROOT, "jni", "java", "org", "dma", "sketchml", "hip", "HipCodec.java")).read()
    natives = set(re.findall(r"static native [\w\[\]]+ (\w+)\(", java))
    c = open(os.path.join(ROOT, "jni", "skml_jni.c")).read()
    exported = set(re.findall(r"Java_org_dma_sketchml_hip_HipCodec_(\w+)\(", c))
    assert natives and natives == exported, (natives ^ exported)


def test_shim_calls_only_declared_entry_points():
    hdr = open(os.path.join(ROOT, "include", "skml.h")).read()
    declared = set(re.findall(r"\b(skml_\w+)\s*\(", hdr))
    c = open(os.path.join(ROOT, "jni", "skml_jni.c")).read()
    used = set(re.findall(r"\b(skml_\w+)\s*\(", c))
    assert used <= declared, used - declared
