"""The two remaining CMake routes to libmchecksum (CMake
contract), each built from source with CMakeLists.txt.  CPU only: hipcc
cross-compiles the gfx950 kernels here, and nothing launches them.

- Bundled mode, the way Mercury builds mchecksum when
  MERCURY_USE_SYSTEM_MCHECKSUM is OFF (reference src/CMakeLists.txt:73-83):
  the parent sets MCHECKSUM_EXTERNALLY_CONFIGURED, the four
  MCHECKSUM_INSTALL_*_DIR and MCHECKSUM_EXTERNAL_EXPORTED_TARGETS, calls
  add_subdirectory, includes ${MCHECKSUM_BINARY_DIR}/mchecksum-config.cmake
  and links the target `mchecksum` privately into its own library
  (src/CMakeLists.txt:192-194).  The parent's install must carry mchecksum in
  its export set.
- Installed system mode: a standalone build installed to a prefix, then found
  by a consumer's find_package(mchecksum REQUIRED) through CMAKE_PREFIX_PATH.

Both consumers run Mercury's init/update/get/destroy sequence
(src/mercury_proc.c:70,398,374,136) on the CRC-32C check string, and they
call one batch entry point of mchecksum_gpu.h to show that it links.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(shutil.which("cmake") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="cmake or hipcc not installed")

# stands in for Mercury's hg_proc layer: a shared library linking mchecksum privately
PROC_C = r"""#include <mchecksum.h>
#include <stdint.h>
int proc_crc32c(const void *a, size_t na, const void *b, size_t nb, uint32_t *out) {
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    if (mchecksum_init("crc32c", &c) != 0) return 2;
    if (mchecksum_get_size(c) != 4) return 6;
    if (mchecksum_update(c, a, na) || mchecksum_update(c, b, nb)) return 3;
    if (mchecksum_get(c, out, sizeof(*out), MCHECKSUM_FINALIZE) != 0) return 4;
    if (mchecksum_destroy(c) != 0 || mchecksum_destroy(MCHECKSUM_OBJECT_NULL) != 0) return 5;
    return 0;
}
"""

MAIN_C = r"""#include <stdint.h>
#include <stdio.h>
int proc_crc32c(const void *, unsigned long, const void *, unsigned long, uint32_t *);
int main(void) {
    uint32_t h = 0;
    int rc = proc_crc32c("12345", 5, "6789", 4, &h);
    if (rc) return rc;
    printf("%08x\n", h);
    return h == 0xE3069283u ? 0 : 1;
}
"""

GPU_C = r"""#include <mchecksum_gpu.h>
#include <stdio.h>
int main(void) { printf("gpu %d\n", mchecksum_gpu_available()); return 0; }
"""

BUNDLED = """cmake_minimum_required(VERSION 3.21)
project(MERCURY C)
set(MERCURY_EXPORTED_TARGETS mercury-targets)
# reference src/CMakeLists.txt:74-83
set(MCHECKSUM_EXTERNALLY_CONFIGURED 1)
set(MCHECKSUM_INSTALL_BIN_DIR bin)
set(MCHECKSUM_INSTALL_LIB_DIR lib)
set(MCHECKSUM_INSTALL_INCLUDE_DIR include)
set(MCHECKSUM_INSTALL_DATA_DIR share)
set(MCHECKSUM_EXTERNAL_EXPORTED_TARGETS ${MERCURY_EXPORTED_TARGETS})
add_subdirectory(%(root)s mchecksum)
include(${MCHECKSUM_BINARY_DIR}/mchecksum-config.cmake)
if(NOT mchecksum_FOUND OR NOT MCHECKSUM_LIBRARIES STREQUAL "mchecksum")
  message(FATAL_ERROR "build-tree mchecksum-config.cmake incomplete")
endif()
add_library(mercury SHARED proc.c)
target_link_libraries(mercury PRIVATE mchecksum)
add_executable(consumer main.c)
target_link_libraries(consumer PRIVATE mercury)
add_executable(gpu_probe gpu.c)
target_link_libraries(gpu_probe PRIVATE mchecksum)
install(TARGETS mercury EXPORT ${MERCURY_EXPORTED_TARGETS} LIBRARY DESTINATION lib)
install(EXPORT ${MERCURY_EXPORTED_TARGETS} DESTINATION share/cmake/mercury)
"""

SYSTEM = """cmake_minimum_required(VERSION 3.21)
project(consumer C)
find_package(mchecksum 2.0 REQUIRED)
add_library(mercury SHARED proc.c)
target_link_libraries(mercury PRIVATE mchecksum)
add_executable(consumer main.c)
target_link_libraries(consumer PRIVATE mercury)
add_executable(gpu_probe gpu.c)
target_link_libraries(gpu_probe PRIVATE mchecksum)
"""


def _run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, **kw)
    assert r.returncode == 0, " ".join(cmd) + "\n" + r.stdout[-3000:] + r.stderr[-3000:]
    return r


def _sources(d):
    (d / "proc.c").write_text(PROC_C)
    (d / "main.c").write_text(MAIN_C)
    (d / "gpu.c").write_text(GPU_C)


def _check_consumer(build):
    r = _run([str(build / "consumer")])
    assert r.stdout.strip() == "e3069283"
    r = _run([str(build / "gpu_probe")])
    assert r.stdout.strip() in ("gpu 0", "gpu 1")


def _jobs():
    return str(min(8, os.cpu_count() or 1))


def test_bundled_add_subdirectory(tmp_path):
    src = tmp_path / "src"
    src.mkdir()
    _sources(src)
    (src / "CMakeLists.txt").write_text(BUNDLED % {"root": ROOT})
    build, prefix = tmp_path / "build", tmp_path / "prefix"
    _run(["cmake", "-S", str(src), "-B", str(build), "-G", "Unix Makefiles", f"-DCMAKE_INSTALL_PREFIX={prefix}"])
    assert (build / "mchecksum" / "mchecksum-config.cmake").exists()
    _run(["cmake", "--build", str(build), "-j", _jobs()])
    _check_consumer(build)
    _run(["cmake", "--install", str(build)])
    assert (prefix / "lib" / "libmchecksum.so.2").exists()
    assert (prefix / "include" / "mchecksum.h").exists() and (prefix / "include" / "mchecksum_gpu.h").exists()
    # mchecksum went into the parent's export set, next to mercury
    exports = "".join(p.read_text() for p in (prefix / "share" / "cmake" / "mercury").glob("mercury-targets*.cmake"))
    assert "add_library(mchecksum SHARED IMPORTED)" in exports and "add_library(mercury SHARED IMPORTED)" in exports


def test_installed_find_package(tmp_path):
    build, prefix = tmp_path / "build", tmp_path / "prefix"
    _run(["cmake", "-S", ROOT, "-B", str(build), "-G", "Unix Makefiles", f"-DCMAKE_INSTALL_PREFIX={prefix}"])
    _run(["cmake", "--build", str(build), "-j", _jobs()])
    _run(["cmake", "--install", str(build)])
    assert (prefix / "share" / "cmake" / "mchecksum" / "mchecksum-config.cmake").exists()
    src = tmp_path / "consumer"
    src.mkdir()
    _sources(src)
    (src / "CMakeLists.txt").write_text(SYSTEM)
    cbuild = tmp_path / "cbuild"
    _run(["cmake", "-S", str(src), "-B", str(cbuild), "-G", "Unix Makefiles", f"-DCMAKE_PREFIX_PATH={prefix}"])
    _run(["cmake", "--build", str(cbuild)])
    _check_consumer(cbuild)
