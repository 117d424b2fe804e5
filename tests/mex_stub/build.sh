#!/bin/bash
# TEST-ONLY: compile matlab/ccsc_mex.c against the mex.h stand-in and link the
# harness (tests/mex_stub/_build/libccsc_mexharness.so) against the in-tree libccsc.
set -e
here=$(cd "$(dirname "$0")" && pwd)
root=$(cd "$here/../.." && pwd)
mkdir -p "$here/_build"
gcc -O1 -std=c11 -Wall -Wextra -Werror -Wno-unused-parameter -fPIC -I"$here" -I"$root/include" \
    -c "$root/matlab/ccsc_mex.c" -o "$here/_build/ccsc_mex.o"
gcc -O1 -std=c11 -D_POSIX_C_SOURCE=200809L -Wall -Werror -fPIC -I"$here" -c "$here/mexstub.c" -o "$here/_build/mexstub.o"
gcc -shared -o "$here/_build/libccsc_mexharness.so" "$here/_build/ccsc_mex.o" "$here/_build/mexstub.o" \
    -L"$root/ccsc_code_iccv2017_amd" -lccsc -Wl,-rpath,"$root/ccsc_code_iccv2017_amd" -Wl,--no-undefined
# the solver gateway (matlab/ccsc_solve_mex.c) gets its own harness: both define mexFunction
gcc -O1 -std=c11 -Wall -Wextra -Werror -Wno-unused-parameter -fPIC -I"$here" -I"$root/include" \
    -c "$root/matlab/ccsc_solve_mex.c" -o "$here/_build/ccsc_solve_mex.o"
gcc -shared -o "$here/_build/libccsc_solvemexharness.so" "$here/_build/ccsc_solve_mex.o" "$here/_build/mexstub.o" \
    -L"$root/ccsc_code_iccv2017_amd" -lccsc -Wl,-rpath,"$root/ccsc_code_iccv2017_amd" -Wl,--no-undefined
echo "$here/_build/libccsc_mexharness.so"
