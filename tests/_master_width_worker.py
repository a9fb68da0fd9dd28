"""Run by tests/test_master_width.py: a plain script whose session asks for ``local-cpu[2]`` SPMD
ranks — started WITHOUT a launcher, the session itself starts the two ranks."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from net.jgp.labs.sparkdq4ml_amd import SparkSession  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.parallel import comm  # noqa: E402

spark = SparkSession.builder().master("local-cpu[2]").config("dq4ml.spmd", "true").getOrCreate()
df = spark.range(10)
print(json.dumps({"rank": comm.rank(), "world": comm.world_size(), "width": spark.defaultParallelism,
                  "count": df.count()}), flush=True)
comm.shutdown()
