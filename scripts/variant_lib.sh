# Build a variant of the library that differs only in the N = 10 register-kernel unit and its host
# dispatch (extra compile definitions or an edited mtg_solve_reg.inc), linked against the main
# build's other objects (run `cmake --build build` first).  Timing A/B of N = 10 only: the other
# N units keep the main build's code.  usage: bash scripts/variant_lib.sh NAME [-DMACRO[=V] ...]
# UNITS: the units to rebuild; SRCDIR: where they (and the .inc they include) are taken from
# (default csrc; e.g. a directory with an older mtg_solve_dl.inc checked out of git).
# Output: mav_trajectory_generation_cmake_amd/lib_var/NAME/libmav_trajectory_generation.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
OBJ=build/CMakeFiles/mav_trajectory_generation.dir/mav_trajectory_generation_cmake_amd/csrc
OUT=mav_trajectory_generation_cmake_amd/lib_var/$name
mkdir -p $OUT
# the N = 10 kernel unit and the register kernels' host dispatch (LDS size), with the definitions
UNITS=${UNITS:-mtg_solve_reg_n10 mtg_solve_reg}  # (another kernel: UNITS="mtg_jacobian_n10")
for u in $UNITS; do
  /opt/rocm/llvm/bin/clang++ -D__HIP_ROCclr__=1 -Dmav_trajectory_generation_EXPORTS -I include \
    -I mav_trajectory_generation_cmake_amd/csrc -O3 -DNDEBUG -std=gnu++17 --offload-arch=gfx950 -fPIC \
    -Wall -Wno-unused-parameter "$@" -o $OUT/$u.o -x hip -c ${SRCDIR:-mav_trajectory_generation_cmake_amd/csrc}/$u.hip
done
excl=""; for u in $UNITS; do excl="$excl -e /$u.hip.o\$"; done
objs=$(ls $OBJ/*.o | grep -v $excl)
/opt/rocm/llvm/bin/clang++ -fPIC -O3 --offload-arch=gfx950 -shared --hip-link --rtlib=compiler-rt -unwindlib=libgcc \
  -Wl,-soname,libmav_trajectory_generation.so -o $OUT/libmav_trajectory_generation.so $objs $(for u in $UNITS; do echo $OUT/$u.o; done)
rm -f $OUT/*.o
echo built $OUT
