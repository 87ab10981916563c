#!/bin/bash
# bash equivalent of train_cpu_mp.csh
if command -v mpiexec >/dev/null 2>&1; then
    mpiexec -n 4 python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich "$@"
else
    python3 -m pytorch_ddp_mnist_amd.parallel.launch -n 4 --style pmi -- \
        python3 mnist_pnetcdf_cpu_mp.py --parallel --wireup_method mpich "$@"
fi
