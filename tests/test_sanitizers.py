"""Host code under sanitizers, on the CPU (GPU AddressSanitizer / XNACK builds are not available on
this pool, so the device kernels are not in these builds):

  - AddressSanitizer + UndefinedBehaviorSanitizer: WAV ingest (csrc/tfp_wav.cpp: every layout, every
    header truncation, random bytes), the DSP tables (csrc/tfp_tables.cpp), the oracle's fingerprint
    and its three searches (oracle/oracle.c, oracle/oracle_boxes.c) — tests/native/sanitize_host.cpp;
    and the SQLite catalog (shim/fp_catalog.c) through its CPU harness, life cycle plus 8 threads.
  - ThreadSanitizer: the device group's shard fan-out (csrc/tfp_shardpool.hpp) and the search
    coalescer (csrc/tfp_coalesce.hpp) from many threads (tests/native/tsan_threads.cpp); the catalog's
    lock from 8 threads racing on the same files (shim/fp_catalog.c, harness command cthreads).

Any sanitizer finding makes the program exit non-zero (halt_on_error / -fno-sanitize-recover)."""
import json
import os
import subprocess
import wave

import numpy as np
import pytest

from conftest import REPO

NATIVE = os.path.join(REPO, "tests", "native")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
ASAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
TSAN = ["-fsanitize=thread", "-g", "-O1"]
CAT_INC = ["-I" + os.path.join(REPO, d) for d in ("shim", "include", "tests/native", "tests/native/asterisk_stub")] + \
    ["-idirafter", "/opt/conda/include"]


def _run(cmd, timeout=600):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=SAN_ENV)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-6000:]
    return r.stdout


def test_host_code_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_host")
    objs = []
    for src in ("oracle.c", "oracle_boxes.c"):
        o = str(tmp_path / (src + ".o"))
        subprocess.run(["gcc", "-std=gnu99", "-ffp-contract=off", "-fno-builtin", *ASAN, "-c",
                        os.path.join(REPO, "oracle", src), "-o", o], check=True)
        objs.append(o)
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", "-fno-builtin", *ASAN, "-I" + os.path.join(REPO, "include"),
                    os.path.join(NATIVE, "sanitize_host.cpp"),
                    os.path.join(REPO, "asterisk-tiresias_amd", "csrc", "tfp_wav.cpp"),
                    os.path.join(REPO, "asterisk-tiresias_amd", "csrc", "tfp_tables.cpp"), *objs, "-o", exe, "-lpthread",
                    "-lm"], check=True)
    assert _run([exe]).strip().endswith("ok")


def test_shard_pool_and_coalescer_tsan(tmp_path):
    exe = str(tmp_path / "tsan_threads")
    subprocess.run(["g++", "-std=c++17", *TSAN, "-I" + os.path.join(REPO, "include"),
                    os.path.join(NATIVE, "tsan_threads.cpp"), "-o", exe, "-lpthread"], check=True)
    out = _run([exe])
    assert out.strip().endswith("ok")


def _wav(path, pcm):
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(8000)
        w.writeframes(np.ascontiguousarray(pcm, np.int16).tobytes())


@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_catalog_under_sanitizers(tmp_path, san):
    """The catalog's life cycle (create, dedup, rows, lists, contexts, delete, backup, reload) under
    ASan + UBSan, and 8 threads creating / storing / reading / deleting on 6 shared files under both:
    of the threads that race on one file, exactly one creates its row at a time."""
    exe = str(tmp_path / ("catalog_" + san))
    subprocess.run(["gcc", "-std=gnu99", "-Wall", *(ASAN if san == "asan" else TSAN), *CAT_INC,
                    os.path.join(REPO, "shim", "fp_catalog.c"), os.path.join(NATIVE, "catalog_harness.c"), "-o", exe,
                    "-l:libsqlite3.so.0", "-lcrypto", "-lm", "-lpthread"], check=True)
    rng = np.random.default_rng(3)
    files = []
    for i in range(6):
        files.append(str(tmp_path / ("f%d.wav" % i)))
        _wav(files[-1], rng.integers(-3000, 3000, 4000 + 17 * i))
    db = str(tmp_path / "cat.db")
    out = [json.loads(l) for l in _run([exe, db, "init", "create", "ctx", files[0], "00000000-0000-4000-8000-000000000001",
                                        "create", "ctx", files[0], "00000000-0000-4000-8000-000000000002", "lists",
                                        "ctx", "c2", str(tmp_path), "ctxdel", "c2",
                                        "cthreads", "8", "40", "6", *files, "lists", "term"]).splitlines()]
    ct = next(o for o in out if "cthreads" in o)
    assert ct["calls"] == 320 and ct["created"] + ct["dup"] == 320 and ct["created"] >= 6
    lists = [o for o in out if "audio_lists" in o]
    assert len(lists[-1]["audio_lists"]) == 1  # only the first create is left: every thread deleted its rows
    assert out[-1] == {"term": True}
    out2 = [json.loads(l) for l in _run([exe, db, "init", "lists", "term"]).splitlines()]
    assert len(next(o for o in out2 if "audio_lists" in o)["audio_lists"]) == 1  # reloaded from the backup
