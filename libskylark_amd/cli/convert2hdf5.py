"""``skylark_convert2hdf5``: LIBSVM -> HDF5 conversion (reference
``ml/skylark_convert2hdf5.cpp``).  Writes through h5py when installed,
otherwise through the built-in HDF5 writer (``io/h5.py``)."""
from __future__ import annotations

import argparse
import sys

from .. import io as IO


def main(argv=None):
    p = argparse.ArgumentParser(prog="skylark_convert2hdf5")
    p.add_argument("inputfile")
    p.add_argument("outputfile")
    p.add_argument("--sparse", action="store_true")
    a = p.parse_args(argv)
    X, Y = IO.read_libsvm(a.inputfile, sparse=a.sparse)
    try:
        IO.write_hdf5(a.outputfile, X, Y)
    except IO.IOError_ as e:
        print(f"error: {e}", file=sys.stderr)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
