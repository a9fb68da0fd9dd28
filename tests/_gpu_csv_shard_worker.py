"""One rank of the 2-process sharded device CSV read in ``test_gpu_distributed.py``: each rank
device-scans its row-aligned byte range of a file with string / quoted / timestamp columns, the
type masks are merged across ranks (X3) and ``collect`` gathers the rows in rank order (X5).
Prints one JSON line (rank 0: every row)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession
    from net.jgp.labs.sparkdq4ml_amd.ops import csvscan
    from net.jgp.labs.sparkdq4ml_amd.parallel import comm

    path = sys.argv[1]
    comm.init(backend="gloo")
    r = comm.rank()
    spark = SparkSession.builder().master("mi355x[*]").config("dq4ml.csv.deviceThresholdBytes", "0").getOrCreate()
    b0, f0 = csvscan.STATS["device_scans"], csvscan.STATS["fallbacks"]
    df = spark.read().option("inferSchema", "true").csv(path)
    dev = csvscan.STATS["device_scans"] - b0
    fb = csvscan.STATS["fallbacks"] - f0
    rows = [[None if v is None else str(v) for v in row] for row in df.collect()]
    print(json.dumps({"rank": r, "types": [t for _, t in df.dtypes], "device_scans": dev, "fallbacks": fb,
                      "rows": rows if r == 0 else len(rows)}))
    comm.barrier()
    comm.shutdown()


if __name__ == "__main__":
    main()
