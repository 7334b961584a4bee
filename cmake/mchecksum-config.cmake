# mchecksum-config.cmake -- lets Mercury find this library in "system" mode:
#   cmake <mercury> -DMERCURY_USE_CHECKSUMS=ON -DMERCURY_USE_SYSTEM_MCHECKSUM=ON \
#         -Dmchecksum_DIR=<this repo>/cmake
# Mercury then runs find_package(mchecksum REQUIRED) and links the target
# `mchecksum` (reference src/CMakeLists.txt:66-72,192-194); downstream
# consumers re-include this file (reference CMake/mercury-config.cmake.in:35-36).
get_filename_component(_MCK_ROOT "${CMAKE_CURRENT_LIST_DIR}/.." ABSOLUTE)
set(MCHECKSUM_INCLUDE_DIRS "${_MCK_ROOT}/include")
set(MCHECKSUM_LIBRARY "${_MCK_ROOT}/mercury_amd/lib/libmchecksum.so")
if(NOT EXISTS "${MCHECKSUM_LIBRARY}")
  message(FATAL_ERROR "mchecksum: ${MCHECKSUM_LIBRARY} not built (run `make` in ${_MCK_ROOT})")
endif()
if(NOT TARGET mchecksum)
  add_library(mchecksum SHARED IMPORTED)
  set_target_properties(mchecksum PROPERTIES
    IMPORTED_LOCATION "${MCHECKSUM_LIBRARY}"
    IMPORTED_SONAME "libmchecksum.so.2"
    INTERFACE_INCLUDE_DIRECTORIES "${MCHECKSUM_INCLUDE_DIRS}")
endif()
set(MCHECKSUM_LIBRARIES mchecksum)
set(mchecksum_FOUND TRUE)
