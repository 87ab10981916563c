#!/bin/csh
# 4 ranks, PnetCDF-format input, MPICH-style wire-up (reference train_cpu_mp.csh).
# No MPI in this image: fall back to the bundled PMI-style launcher.
which mpiexec >& /dev/null
if ( $status == 0 ) then
    mpiexec -n 4 python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich $argv
else
    python3 -m pytorch_ddp_mnist_amd.parallel.launch -n 4 --style pmi -- python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich $argv
endif
