"""Cluster benchmark drivers (SURVEY.md §2.12 "Benchmarks"): generated Spark scripts and
commands, and the parsers on the result formats the reference's READMEs document."""
from cloudtik_amd.benchmarks import HiBench, KafkaBench, SparkTPCDS, SQLEnginePowerTest, TPCxAI

THROUGHPUT_OUT = """stream_0 has finished.
+----------+------------------+
|    stream|      sum(Runtime)|
+----------+------------------+
|  stream_0|441.92720381699996|
|  stream_1|     394.519159437|
|max_stream|441.92720381699996|
+----------+------------------+
"""

TPCX_OUT = """========== RESULTS ==========
phase_name  Phase.SERVING_1  Phase.TRAINING_1
use_case
2                   153.826           430.651
5                    91.367           200.453
9                    93.398           246.164
"""


def test_tpcds_scripts_and_commands(tmp_path):
    b = SparkTPCDS(scale_factor=100, fsdir="s3a://bucket", iterations=2)
    paths = b.write_scripts(str(tmp_path))
    assert set(paths) == {"tpcds-datagen.scala", "tpcds-power-test.scala", "tpcds-throughput-test.scala"}
    assert "genData" in open(paths["tpcds-datagen.scala"]).read()
    assert "streamNumber" in open(paths["tpcds-throughput-test.scala"]).read()
    cmd = b.submit_command("c.yaml", paths["tpcds-throughput-test.scala"], streams=4)
    assert cmd[:3] == ["cloudtik", "submit", "c.yaml"] and "spark.driver.streamNumber=4" in cmd
    assert "spark.driver.scaleFactor=100" in cmd and "--jars" in cmd
    assert b.database == "tpcds_parquet_100"
    s = SparkTPCDS.parse_stream_summary(THROUGHPUT_OUT)
    assert s == {"stream_0": 441.92720381699996, "stream_1": 394.519159437, "max_stream": 441.92720381699996}


def test_tpcx_ai_template_command_and_results():
    t = TPCxAI()
    assert t.fill_template("threads: {%Case09_TF_NUM_INTRAOP_THREADS%}", {"Case09_TF_NUM_INTRAOP_THREADS": 16}) \
        == "threads: 16"
    assert "--phase {TRAINING,SERVING}" in t.run_command() and "-uc {2,5,9}" in t.run_command()
    r = TPCxAI.parse_results(TPCX_OUT)
    assert r[2] == {"Phase.SERVING_1": 153.826, "Phase.TRAINING_1": 430.651} and r[9]["Phase.TRAINING_1"] == 246.164


def test_hibench_kafka_sql_engines():
    h = HiBench()
    confs = h.confs("yarn", 4, 8, "16g", "hdfs://head:9000")
    assert "hibench.yarn.executor.num       4" in confs["spark.conf"] and "hdfs://head:9000" in confs["hadoop.conf"]
    assert h.run_commands("ml/kmeans")[1].endswith("ml/kmeans/spark/run.sh")
    rows = HiBench.parse_report("Type Date Time Input_data_size Duration(s) Throughput(bytes/s) Throughput/node\n"
                                "ScalaSparkKmeans 2024-01-01 10:00:00 3991293 42.1 94800 23700\n")
    assert rows == [{"type": "ScalaSparkKmeans", "input_bytes": 3991293, "duration_s": 42.1,
                     "throughput_bytes_s": 94800.0}]
    k = KafkaBench("head:9092")
    assert "kafka-producer-perf-test.sh" in k.commands()[1]
    p = KafkaBench.parse_producer("5000000 records sent, 812345.6 records/sec (77.47 MB/sec), 12.3 ms avg latency, "
                                  "300.0 ms max latency, ...")
    assert p["records_per_sec"] == 812345.6 and p["mb_per_sec"] == 77.47
    cmds = SQLEnginePowerTest("trino", "head:8081").power_commands("/q", 3)
    assert len(cmds) == 3 and cmds[0].startswith("trino --server head:8081 --catalog tpcds")


def test_cli_prints_command(tmp_path, capsys):
    from cloudtik_amd.benchmarks.cluster_bench import main
    assert main(["tpcds", "power", "--cluster", "x.yaml", "--out-dir", str(tmp_path)]) == 0
    out = capsys.readouterr().out
    assert "cloudtik submit x.yaml" in out and "tpcds-power-test.scala" in out
