"""``python -m test_nccl_p2p_amd [p2p_matrix options]``

Runs the native p2p_matrix application in-process.  Under ``torchrun`` the
ranks bootstrap over TCP from RANK / WORLD_SIZE / MASTER_ADDR (port
MASTER_PORT+1 or P2P_BOOTSTRAP_PORT); alone it is a single rank (self path).
``mpirun -n N ./build/p2p_matrix`` is the MPI-launched equivalent.
"""

import sys

from . import require_native


def main(argv=None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    return int(require_native().run_cli(args))


if __name__ == "__main__":
    sys.exit(main())
