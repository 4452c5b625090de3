# Build a variant of the library that differs only in the N = 10 register-kernel unit (extra
# compile definitions), linked against the main build's other objects (run `cmake --build build`
# first).  usage: bash scripts/variant_lib.sh NAME [-DMACRO[=V] ...]
# Output: mav_trajectory_generation_cmake_amd/lib_var/NAME/libmav_trajectory_generation.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
OBJ=build/CMakeFiles/mav_trajectory_generation.dir/mav_trajectory_generation_cmake_amd/csrc
OUT=mav_trajectory_generation_cmake_amd/lib_var/$name
mkdir -p $OUT
/opt/rocm/llvm/bin/clang++ -D__HIP_ROCclr__=1 -Dmav_trajectory_generation_EXPORTS -I include \
  -I mav_trajectory_generation_cmake_amd/csrc -O3 -DNDEBUG -std=gnu++17 --offload-arch=gfx950 -fPIC \
  -Wall -Wno-unused-parameter "$@" -o $OUT/n10.o -x hip -c mav_trajectory_generation_cmake_amd/csrc/mtg_solve_reg_n10.hip
objs=$(ls $OBJ/*.o | grep -v '/mtg_solve_reg_n10.hip.o$')
/opt/rocm/llvm/bin/clang++ -fPIC -O3 --offload-arch=gfx950 -shared --hip-link --rtlib=compiler-rt -unwindlib=libgcc \
  -Wl,-soname,libmav_trajectory_generation.so -o $OUT/libmav_trajectory_generation.so $objs $OUT/n10.o
rm -f $OUT/n10.o
echo built $OUT
