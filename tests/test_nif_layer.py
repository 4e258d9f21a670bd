"""The pure-C half of the vmq_reg_gpu_view NIF (integration/c_src/vmqg_batch.c):
compiled with gcc against include/vmqg.h and libvmqgpu.so, and run over a
host-engine-only context (no GPU): interners, subscription ops from filter
strings, publish batches (vmq_topic:validate_topic splitting, rejection,
growth, merging per-thread batches), the fold over records and over ranges,
and the loud refusal to match without a device."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_batch_layer_unit(tmp_path):
    from vernemq_amd import _lib
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    exe = tmp_path / "test_batch"
    subprocess.run(["gcc", "-std=c99", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "integration", "c_src"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "c", "test_batch.c"),
                    os.path.join(ROOT, "integration", "c_src", "vmqg_batch.c"),
                    "-L", lib_dir, "-l:libvmqgpu.so", "-Wl,-rpath," + lib_dir], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_nif_sources_are_present():
    """The Erlang drop-in and its NIF glue ship as files (OTP is not in this
    image: they are not compiled here; their C core above is)."""
    erl = open(os.path.join(ROOT, "integration", "src", "vmq_reg_gpu_view.erl")).read()
    nif = open(os.path.join(ROOT, "integration", "c_src", "vmqg_nif.c")).read()
    for needle in ("-behaviour(vmq_reg_view)", "fold(", "start_link()", "stats()", "subscribe_subscriber_changes"):
        assert needle in erl, needle
    for needle in ("ERL_NIF_INIT", "vmqgb_match", "vmqgb_fold", "vmqgb_ops_apply", "ERL_NIF_DIRTY_JOB_CPU_BOUND"):
        assert needle in nif, needle
