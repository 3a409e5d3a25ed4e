#!/bin/bash
# Test infrastructure only: build the CPU SIMT emulation of the decode kernel (tests/emu/_build).
# The kernel source is compiled as host C++ against tests/emu/hip/hip_runtime.h; the two
# device-only spellings it uses (address-space qualifiers, the in-place kernarg read, the vmcnt wait) are rewritten on the
# way in. Nothing here is linked into libkxcodec.so.
set -e
cd "$(dirname "$0")"
ROOT=../..
OUT=${EMU_OUT:-_build}
mkdir -p $OUT
sed -e 's/^#define LDS __attribute__((address_space(3)))/#define LDS/' \
    -e 's/^#define GLB __attribute__((address_space(1)))/#define GLB/' \
    -e 's/^#define KAS __attribute__((address_space(4))).*/#define KAS/' \
    -e 's/^#define KX_PARAMS() .*/#define KX_PARAMS() (dp_)/' \
    -e 's/__attribute__((amdgpu_waves_per_eu([0-9]*))) //' \
    -e 's/asm volatile("s_waitcnt vmcnt(0)" ::: "memory");/emu_wait_vmcnt0();/' \
    -e 's/asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");/emu_wait_vmcnt0();/' \
    -e 's/asm volatile("s_mov_b32 %0, 0" : "=s"(z));/z = 0;/' \
    -e 's|^  return \*(const GLB uint32_t\*)A;  // input tail dword$|  return emu_gdword(A, end);|' \
    $ROOT/kitex_amd/csrc/kx_decode.hip > $OUT/kx_decode_emu.cpp
CXX=${CXX:-/opt/rocm/lib/llvm/bin/clang++}
FLAGS="-std=c++17 -O1 -g -fPIC -Wno-unknown-attributes -Wno-unused-function -I. -I$ROOT/kitex_amd/csrc ${EMU_EXTRA:-}"
$CXX $FLAGS -c $OUT/kx_decode_emu.cpp -o $OUT/kx_decode_emu.o
cp $ROOT/kitex_amd/csrc/kx_crc.hip $OUT/kx_crc_emu.cpp
$CXX $FLAGS -c $OUT/kx_crc_emu.cpp -o $OUT/kx_crc_emu.o
$CXX $FLAGS -c $ROOT/kitex_amd/csrc/kx_schema.cpp -o $OUT/kx_schema.o
$CXX $FLAGS -c $ROOT/kitex_amd/csrc/kx_knobs.cpp -o $OUT/kx_knobs.o
$CXX $FLAGS -c $ROOT/kitex_amd/csrc/kx_nested_schema.cpp -o $OUT/kx_nested_schema.o
$CXX $FLAGS -c nested_host.cpp -o $OUT/nested_host.o
$CXX $FLAGS -c emu_rt.cpp -o $OUT/emu_rt.o
$CXX $FLAGS -c emu_driver.cpp -o $OUT/emu_driver.o
$CXX -shared -o $OUT/libkxemu.so $OUT/*.o -lpthread
echo $OUT/libkxemu.so
