"""HDFS, YARN and Spark runtimes that configure themselves (reference runtime/hdfs,
runtime/yarn, runtime/spark: configure.sh + conf templates + utils.py).

Each runtime renders its Hadoop / Spark configuration files from the templates in
``conf/`` at ``cloudtik runtime configure <name>`` time, from three inputs:

* the cluster-level decisions made once in ``prepare_config`` and exported to every node as
  environment variables (Spark executor sizing, YARN memory ratio, HDFS replication);
* the node itself (head address, CPU count, memory, attached data disks);
* the runtime's config section (``runtime.hdfs`` / ``runtime.yarn`` / ``runtime.spark``).

The YARN runtime also contributes the ``scaling-with-yarn`` scaling policy (ResourceManager
cluster metrics -> resource demands) and the YARN job waiter (wait until no application is
pending or running); the Spark runtime turns ``cloudtik submit job.py|.jar|.scala`` into
``spark-submit`` / ``spark-shell`` commands.
"""
from .runtimes import (HadoopRuntime, HdfsRuntime, SparkRuntime, YarnRuntime,  # noqa: F401
                       spark_executor_resource, yarn_node_resource)
from .yarn import YarnJobWaiter, YarnScalingPolicy  # noqa: F401
