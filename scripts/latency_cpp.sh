# Build and run scripts/latency_cpp.cpp (host only; needs the built library and oracle/mtg_oracle.c).
set -e
cd "$(dirname "$0")/.."
mkdir -p build
gcc -O3 -march=native -ffp-contract=off -std=c99 -c -o build/oracle_lat.o oracle/mtg_oracle.c -I oracle
g++ -O3 -march=native -std=c++17 -o build/latency_cpp scripts/latency_cpp.cpp build/oracle_lat.o -I include -I oracle \
    -L mav_trajectory_generation_cmake_amd/lib -lmav_trajectory_generation \
    -Wl,-rpath,$PWD/mav_trajectory_generation_cmake_amd/lib -lm
MTG_EXECUTION=auto ./build/latency_cpp
