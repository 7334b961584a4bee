"""The CMake package contract Mercury relies on in system mode
(reference src/CMakeLists.txt:62-85: find_package(mchecksum REQUIRED), then
link the imported target `mchecksum`): a minimal consumer project configures
against cmake/mchecksum-config.cmake, builds, links libmchecksum.so and runs
Mercury's init/update/get/destroy sequence (src/mercury_proc.c:70,398,374,136)
on the CRC-32C check string.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CMAKELISTS = """cmake_minimum_required(VERSION 3.10)
project(mchecksum_consumer C)
find_package(mchecksum REQUIRED)
add_executable(consumer consumer.c)
target_link_libraries(consumer PRIVATE mchecksum)
"""

CONSUMER = r"""#include <mchecksum.h>
#include <stdint.h>
#include <stdio.h>
int main(void) {
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    uint32_t h = 0;
    if (mchecksum_init("crc32c", &c) != 0) return 2;
    if (mchecksum_update(c, "12345", 5) || mchecksum_update(c, "6789", 4)) return 3;
    if (mchecksum_get(c, &h, sizeof(h), MCHECKSUM_FINALIZE) != 0) return 4;
    if (mchecksum_destroy(c) != 0 || mchecksum_destroy(MCHECKSUM_OBJECT_NULL) != 0) return 5;
    printf("%08x\n", h);
    return h == 0xE3069283u ? 0 : 1;
}
"""


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")
def test_find_package_consumer_links_and_runs(product_lib, tmp_path):
    (tmp_path / "CMakeLists.txt").write_text(CMAKELISTS)
    (tmp_path / "consumer.c").write_text(CONSUMER)
    build = tmp_path / "build"
    env = dict(os.environ)
    subprocess.run(["cmake", "-S", str(tmp_path), "-B", str(build), "-G", "Unix Makefiles",
                    f"-Dmchecksum_DIR={os.path.join(ROOT, 'cmake')}"], check=True, capture_output=True, env=env)
    subprocess.run(["cmake", "--build", str(build)], check=True, capture_output=True, env=env)
    r = subprocess.run([str(build / "consumer")], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "e3069283"


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not installed")
def test_batch_abi_consumer_builds_through_the_package(product_lib, tmp_path):
    """The batch path's C binding (tests/native/hg_verify_consumer.c, the
    INTEGRATION.md section 3 consumer) includes <mchecksum_gpu.h>, finds the
    library through cmake/mchecksum-config.cmake, compiles with -Werror and
    links libmchecksum + the HIP runtime.  On this GPU-less box it must see
    every entry point refuse with MCHECKSUM_GPU_ENODEV (no host fallback);
    tests/test_gpu_consumer.py runs the same program on the MI355X."""
    build = tmp_path / "build"
    src = os.path.join(ROOT, "tests", "native", "hg_consumer")
    subprocess.run(["cmake", "-S", src, "-B", str(build), f"-Dmchecksum_DIR={os.path.join(ROOT, 'cmake')}"],
                   check=True, capture_output=True)
    subprocess.run(["cmake", "--build", str(build)], check=True, capture_output=True)
    r = subprocess.run([str(build / "hg_verify_consumer")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("NODEV"), r.stdout


def test_batch_abi_consumer_is_built_in_tree():
    """`make` leaves the consumer at build/hg_verify_consumer for the GPU box,
    which runs the tree without building."""
    assert os.access(os.path.join(ROOT, "build", "hg_verify_consumer"), os.X_OK), "run make"
