"""Self-configuring HDFS / YARN / Spark / Hadoop-client runtimes.

Reference behaviour reproduced (not its bash): runtime/hdfs/scripts/configure.sh + hdfs.sh
(name / data dirs on the data disks, one-time namenode format), runtime/yarn/scripts/
configure.sh (NodeManager memory = node memory x ratio rounded to GB, vcores, scheduler,
local dirs), runtime/spark/utils.py:102-156 (executor cores / memory sizing from the worker
node type) and :170-179 (``spark-submit`` / ``spark-shell`` runnable commands).
"""
from __future__ import annotations

import getpass
import glob
import os
from typing import Any, Dict, List, Optional

from cloudtik_amd.runtime.catalog import SPEC_BY_NAME, CatalogRuntime
from cloudtik_amd.runtime.hadoop import cloud_storage
from cloudtik_amd.runtime.common.runtime_base import render_conf_file

CONF_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "conf")
DATA_DISK_GLOB = "/mnt/cloudtik/data_disk_*"
HDFS_RPC_PORT = 8020
HDFS_HTTP_PORT = 9870

# Spark executor sizing constants (reference runtime/spark/utils.py:26-37)
YARN_MEMORY_RATIO = 0.8
EXECUTOR_CORES = 4
EXECUTOR_CORES_SINGLE_BOUND = 8
DRIVER_MEMORY_RATIO = 0.1
APP_MASTER_MEMORY_RATIO = 0.02
DRIVER_MEMORY_MIN, DRIVER_MEMORY_MAX = 1024, 8192
ADDITIONAL_OVERHEAD = 1024
EXECUTOR_OVERHEAD_MIN, EXECUTOR_OVERHEAD_RATIO = 384, 0.1


def round_gb(mb: float) -> int:
    """Round a MB size down to whole GB, at least 1 GB (in MB)."""
    return max(1, int(mb) // 1024) * 1024


def _clamp(v, lo, hi):
    return max(lo, min(v, hi))


def spark_executor_resource(worker_cpu: int, worker_memory_mb: float, head_memory_mb: float,
                            yarn_memory_ratio: float = YARN_MEMORY_RATIO) -> Dict[str, int]:
    """Executor cores / memory and driver memory (MB) for one worker node type.

    Cores per executor default to 4; small nodes (<= 8 CPUs) run one executor over all of
    them, 9-16 CPUs two executors (rounding an odd count up by one), larger counts that are
    not a multiple of 4 are rounded up to one.  The YARN share of the worker's memory, minus
    an application master and a fixed overhead, is divided between the executors, and each
    executor keeps max(10%, 384 MB) for its off-heap overhead."""
    cpus = int(worker_cpu)
    cores = EXECUTOR_CORES
    if cores > cpus:
        cores = cpus
    elif cpus % EXECUTOR_CORES:
        if cpus <= EXECUTOR_CORES_SINGLE_BOUND:
            cores = cpus
        elif cpus <= 2 * EXECUTOR_CORES_SINGLE_BOUND:
            cpus += cpus % 2
            cores = cpus // 2
        else:
            cpus += EXECUTOR_CORES - cpus % EXECUTOR_CORES
    cores = max(1, cores)
    executors = max(1, cpus // cores)
    yarn_mem = round_gb(worker_memory_mb * yarn_memory_ratio)
    app_master = _clamp(round_gb(yarn_mem * APP_MASTER_MEMORY_RATIO), DRIVER_MEMORY_MIN, DRIVER_MEMORY_MAX)
    overhead = round_gb(app_master + ADDITIONAL_OVERHEAD)
    per_executor = round_gb((yarn_mem - overhead) / executors)
    executor_mem = per_executor - max(int(per_executor * EXECUTOR_OVERHEAD_RATIO), EXECUTOR_OVERHEAD_MIN)
    driver = _clamp(round_gb(head_memory_mb * DRIVER_MEMORY_RATIO), DRIVER_MEMORY_MIN, DRIVER_MEMORY_MAX)
    return {"spark_driver_memory": driver, "spark_executor_cores": cores, "spark_executor_memory": executor_mem}


def yarn_node_resource(cpus: int, memory_mb: float, ratio: float = YARN_MEMORY_RATIO,
                       container_max: Optional[Dict[str, Any]] = None) -> Dict[str, int]:
    """NodeManager resources: memory = node memory x ratio rounded down to GB, all vcores;
    optional ``yarn_container_maximum`` {memory, vcores} caps the per-container maximum."""
    mem = round_gb(memory_mb * ratio)
    out = {"memory_mb": mem, "vcores": int(cpus), "max_alloc_mb": mem, "max_alloc_vcores": int(cpus)}
    if container_max:
        out["max_alloc_mb"] = int(container_max.get("memory", mem))
        out["max_alloc_vcores"] = int(container_max.get("vcores", cpus))
    return out


def _mb(value) -> float:
    """Node-type ``memory`` resource -> MB (bytes if large, else GB/MB heuristics)."""
    v = float(value)
    if v > 1 << 24:          # bytes
        return v / (1 << 20)
    if v < 4096:             # GB
        return v * 1024
    return v


def _node_types(config: Dict[str, Any]):
    types = config.get("available_node_types") or {}
    head_t = config.get("head_node_type")
    head = (types.get(head_t) or {}).get("resources") or {}
    workers = [t for n, t in types.items() if n != head_t]
    worker = ((workers[0] if workers else types.get(head_t)) or {}).get("resources") or head
    return head, worker


def _data_dirs(sub: str, fallback: str) -> str:
    disks = sorted(glob.glob(DATA_DISK_GLOB))
    if disks:
        return ",".join(os.path.join(d, sub) for d in disks)
    return fallback


class _HadoopFamily(CatalogRuntime):
    """Common pieces: one Hadoop installation at $RUNTIME_PATH/hadoop shared by the hadoop /
    hdfs / yarn runtimes, conf rendering from templates at configure time."""

    home_dir = "hadoop"
    home_env = "HADOOP_HOME"
    templates: Dict[str, str] = {}          # template -> path under the conf dir

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        env[self.home_env] = f"$RUNTIME_PATH/{self.home_dir}"
        return env

    def install_steps(self, head):
        s = self.spec
        if not s.download:
            return []
        url = s.download.format(version=s.version)
        dest = f"$RUNTIME_PATH/{self.home_dir}"
        return [f"mkdir -p $RUNTIME_PATH && ( [ -d {dest}/bin ] || ( wget -q -O /tmp/{self.home_dir}.tgz {url} && "
                f"mkdir -p {dest} && tar -xf /tmp/{self.home_dir}.tgz -C {dest} --strip-components=1 ) )"]

    # ---------------------------------------------------------------- configure
    def node_facts(self, head: bool, env: Dict[str, str]) -> Dict[str, Any]:
        import psutil
        head_ip = env.get("CLOUDTIK_HEAD_IP") or (env.get("CLOUDTIK_NODE_IP") if head else None) or "localhost"
        return {"head": head, "head_ip": head_ip, "runtime_path": env.get("RUNTIME_PATH", ""),
                "home": os.path.join(env.get("RUNTIME_PATH", ""), self.home_dir),
                "cpus": int(env.get("CLOUDTIK_NODE_CPUS") or os.cpu_count() or 1),
                "memory_mb": float(env.get("CLOUDTIK_NODE_MEMORY_MB") or psutil.virtual_memory().total / (1 << 20)),
                "user": env.get("USER") or getpass.getuser()}

    def conf_dir(self, facts) -> str:
        return os.path.join(facts["home"], "etc", "hadoop")

    def conf_values(self, facts, env) -> Dict[str, Any]:
        return {}

    def render(self, head: bool) -> Dict[str, str]:
        """Render every template of this runtime for this node; returns {dst: text-path}."""
        env = self.node_env(head)
        facts = self.node_facts(head, env)
        values = self.conf_values(facts, env)
        out = {}
        for tpl, dst in self.templates.items():
            path = os.path.join(self.conf_dir(facts), dst)
            render_conf_file(os.path.join(CONF_DIR, tpl), path, values)
            out[tpl] = path
        return out

    def node_configure(self, head: bool):
        self.render(head)
        return self._run_steps(self.configure_steps(head), head)

    def configure_steps(self, head):
        return [f"mkdir -p $RUNTIME_PATH/{self.home_dir}/logs"]


def _proxyuser(user: str) -> str:
    return "\n".join(f"  <property><name>hadoop.proxyuser.{user}.{k}</name><value>*</value></property>"
                     for k in ("hosts", "groups"))


def _credential_file(facts) -> str:
    return os.path.join(facts["home"], "etc", "hadoop", cloud_storage.CREDENTIAL_STORE)


def _core_values(facts, env, default_fs: str) -> Dict[str, Any]:
    props, secrets = cloud_storage.cloud_storage_conf(env)
    return {"fs.default.name": default_fs,
            "hadoop.tmp.dir": os.path.join(facts["home"], "tmp"),
            "hadoop.proxyuser.properties": _proxyuser(facts["user"]),
            "cloud.storage.properties": cloud_storage.properties_xml(
                props, _credential_file(facts) if secrets else "")}


def _credential_steps(runtime, head) -> List[str]:
    """Secrets of the cloud storage connector into the JCEKS store core-site points at."""
    env = runtime.node_env(head)
    secret_vars = cloud_storage.cloud_storage_secret_vars(env)
    facts = runtime.node_facts(head, env)
    return cloud_storage.credential_commands(secret_vars, facts["home"], _credential_file(facts))


class HadoopRuntime(_HadoopFamily):
    """Hadoop client configuration: fs.defaultFS from the cluster's HDFS, a discovered
    workspace HDFS, or ``runtime.hadoop.default_storage``; cloud connectors use it."""
    spec = SPEC_BY_NAME["hadoop"]
    templates = {"core-site.xml": "core-site.xml"}

    def conf_values(self, facts, env):
        fs = (env.get("HADOOP_DEFAULT_FS") or env.get("HDFS_NAMENODE_URI")
              or cloud_storage.cloud_storage_uri(env) or f"file://{facts['home']}/data")
        return _core_values(facts, env, fs)

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        env.update(cloud_storage.export_cloud_storage_env((config or {}).get("provider", {})))
        rc = (config or {}).get("runtime", {}).get("hadoop", {}) or {}
        if rc.get("default_storage"):
            env["HADOOP_DEFAULT_FS"] = str(rc["default_storage"])
        return env

    def configure_steps(self, head):
        return super().configure_steps(head) + _credential_steps(self, head)


class HdfsRuntime(_HadoopFamily):
    spec = SPEC_BY_NAME["hdfs"]
    templates = {"core-site.xml": "core-site.xml", "hdfs-site.xml": "hdfs-site.xml"}

    def prepare_config(self, cluster_config):
        rc = cluster_config.setdefault("runtime", {}).setdefault("hdfs", {}) or {}
        cluster_config["runtime"]["hdfs"] = rc
        if "dfs_replication" not in rc:
            workers = int(cluster_config.get("min_workers") or 0)
            for name, t in (cluster_config.get("available_node_types") or {}).items():
                if name != cluster_config.get("head_node_type"):
                    workers = max(workers, int(t.get("min_workers") or 0))
            rc["dfs_replication"] = max(1, min(3, workers))
        return cluster_config

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        env.update(cloud_storage.export_cloud_storage_env((config or {}).get("provider", {})))
        rc = (config or {}).get("runtime", {}).get("hdfs", {}) or {}
        env["HDFS_DFS_REPLICATION"] = str(rc.get("dfs_replication", 1))
        env["HDFS_DFS_BLOCKSIZE"] = str(rc.get("dfs_blocksize", 268435456))
        return env

    def name_dir(self, facts) -> str:
        return os.path.join(facts["home"], "data", "dfs", "namenode")

    def conf_values(self, facts, env):
        head = facts["head_ip"]
        vals = _core_values(facts, env, f"hdfs://{head}:{HDFS_RPC_PORT}")
        vals.update({
            "dfs.replication": env.get("HDFS_DFS_REPLICATION", "1"),
            "dfs.blocksize": env.get("HDFS_DFS_BLOCKSIZE", "268435456"),
            "dfs.namenode.name.dir": self.name_dir(facts),
            "dfs.datanode.data.dir": _data_dirs("dfs/data", os.path.join(facts["home"], "data", "dfs", "data")),
            "dfs.namenode.rpc-address": f"{head}:{HDFS_RPC_PORT}",
            "dfs.namenode.http-address": f"{head}:{HDFS_HTTP_PORT}",
        })
        return vals

    def configure_steps(self, head):
        return super().configure_steps(head) + _credential_steps(self, head)

    def start_steps(self, head):
        if not head:
            return ["$HADOOP_HOME/bin/hdfs --daemon start datanode"]
        nn = "$RUNTIME_PATH/hadoop/data/dfs/namenode"
        # format once: the name directory keeps its VERSION file across restarts
        return [f"[ -f {nn}/current/VERSION ] || $HADOOP_HOME/bin/hdfs --loglevel WARN namenode -format "
                f"-force -nonInteractive",
                "$HADOOP_HOME/bin/hdfs --daemon start namenode"]


class YarnRuntime(_HadoopFamily):
    spec = SPEC_BY_NAME["yarn"]
    templates = {"yarn-site.xml": "yarn-site.xml"}

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        rc = (config or {}).get("runtime", {}).get("yarn", {}) or {}
        env["YARN_RESOURCE_MEMORY_RATIO"] = str(rc.get("yarn_resource_memory_ratio", YARN_MEMORY_RATIO))
        env["YARN_SCHEDULER"] = str(rc.get("yarn_scheduler", "capacity"))
        cm = rc.get("yarn_container_maximum") or {}
        if cm.get("memory"):
            env["YARN_CONTAINER_MAXIMUM_MEMORY"] = str(cm["memory"])
        if cm.get("vcores"):
            env["YARN_CONTAINER_MAXIMUM_VCORES"] = str(cm["vcores"])
        return env

    def conf_values(self, facts, env):
        cm = {}
        if env.get("YARN_CONTAINER_MAXIMUM_MEMORY"):
            cm["memory"] = env["YARN_CONTAINER_MAXIMUM_MEMORY"]
        if env.get("YARN_CONTAINER_MAXIMUM_VCORES"):
            cm["vcores"] = env["YARN_CONTAINER_MAXIMUM_VCORES"]
        r = yarn_node_resource(facts["cpus"], facts["memory_mb"],
                               float(env.get("YARN_RESOURCE_MEMORY_RATIO", YARN_MEMORY_RATIO)), cm or None)
        sched = {"fair": "org.apache.hadoop.yarn.server.resourcemanager.scheduler.fair.FairScheduler"}.get(
            env.get("YARN_SCHEDULER", "capacity"),
            "org.apache.hadoop.yarn.server.resourcemanager.scheduler.capacity.CapacityScheduler")
        return {"yarn.resourcemanager.hostname": facts["head_ip"],
                "yarn.resourcemanager.scheduler.class": sched,
                "yarn.nodemanager.resource.memory-mb": r["memory_mb"],
                "yarn.nodemanager.resource.cpu-vcores": r["vcores"],
                "yarn.scheduler.maximum-allocation-mb": r["max_alloc_mb"],
                "yarn.scheduler.maximum-allocation-vcores": r["max_alloc_vcores"],
                "yarn.nodemanager.local-dirs": _data_dirs("yarn/local",
                                                          os.path.join(facts["home"], "data", "yarn", "local")),
                "yarn.nodemanager.resource-plugins": ""}

    def get_scaling_policy(self, cluster_config, head_ip):
        from .yarn import YarnScalingPolicy
        rc = (cluster_config.get("runtime", {}).get("yarn") or {}).get("scaling") or {}
        if rc.get("scaling_mode", "none") in (None, "", "none"):
            return None
        return YarnScalingPolicy(cluster_config, head_ip)

    def get_job_waiter(self, cluster_config):
        from .yarn import YarnJobWaiter
        return YarnJobWaiter(cluster_config)


class SparkRuntime(_HadoopFamily):
    spec = SPEC_BY_NAME["spark"]
    home_dir = "spark"
    home_env = "SPARK_HOME"
    templates = {"spark-defaults.conf": "spark-defaults.conf"}

    def conf_dir(self, facts):
        return os.path.join(facts["home"], "conf")

    def install_steps(self, head):
        s = self.spec
        url = s.download.format(version=s.version)
        return [f"mkdir -p $RUNTIME_PATH && ( [ -d $RUNTIME_PATH/spark/bin ] || ( wget -q -O /tmp/spark.tgz {url} && "
                "mkdir -p $RUNTIME_PATH/spark && tar -xf /tmp/spark.tgz -C $RUNTIME_PATH/spark --strip-components=1 ) )"]

    def prepare_config(self, cluster_config):
        """Size executors once for the cluster from the worker node type (exported to nodes)."""
        head, worker = _node_types(cluster_config)
        runtime = cluster_config.setdefault("runtime", {})
        rc = runtime.get("spark") or {}
        runtime["spark"] = rc
        ratio = float((runtime.get("yarn") or {}).get("yarn_resource_memory_ratio", YARN_MEMORY_RATIO))
        if worker.get("CPU") and worker.get("memory"):
            rc["spark_executor_resource"] = spark_executor_resource(
                int(worker["CPU"]), _mb(worker["memory"]), _mb(head.get("memory", worker["memory"])), ratio)
        return cluster_config

    def with_environment_variables(self, config, provider, node_id):
        env = super().with_environment_variables(config, provider, node_id)
        runtime = (config or {}).get("runtime", {}) or {}
        rc = runtime.get("spark", {}) or {}
        er = rc.get("spark_executor_resource") or {}
        for k, v in er.items():
            env[k.upper()] = str(v)
        types = runtime.get("types") or []
        env["SPARK_WITH_HDFS"] = "true" if "hdfs" in types else "false"
        env["HADOOP_HOME"] = "$RUNTIME_PATH/hadoop"
        env["HADOOP_CONF_DIR"] = "$RUNTIME_PATH/hadoop/etc/hadoop"
        if rc.get("hive_metastore_uri"):
            env["SPARK_METASTORE_URI"] = str(rc["hive_metastore_uri"])
        # SQL optimizations (runtime/hadoop/spark_optimizations.py) and user properties
        # (runtime.spark.config), rendered into spark-defaults.conf on every node
        from cloudtik_amd.runtime.hadoop.spark_optimizations import render_properties, spark_optimization_properties
        opt = spark_optimization_properties(self.spec.version, rc.get("optimizations"),
                                            bool(rc.get("optimized_build", False)))
        lines = [ln for ln in render_properties(opt).split("\n") if ln]
        lines += [f"{k:<38} {v}" for k, v in (rc.get("config") or {}).items()]
        env["SPARK_EXTRA_PROPERTIES"] = ";;".join(lines)     # one line in the exported environment
        return env

    def conf_values(self, facts, env):
        hdfs = env.get("SPARK_WITH_HDFS") == "true"
        base = f"hdfs://{facts['head_ip']}:{HDFS_RPC_PORT}/shared" if hdfs else f"file://{facts['home']}/shared"
        ms = env.get("SPARK_METASTORE_URI")
        return {"spark.driver.memory": f"{env.get('SPARK_DRIVER_MEMORY', 1024)}m",
                "spark.executor.cores": env.get("SPARK_EXECUTOR_CORES", 1),
                "spark.executor.memory": f"{env.get('SPARK_EXECUTOR_MEMORY', 1024)}m",
                "spark.local.dir": _data_dirs("spark/local", os.path.join(facts["home"], "local")),
                "spark.eventLog.dir": f"{base}/spark-events",
                "spark.sql.warehouse.dir": f"{base}/spark-warehouse",
                "spark.hadoop.hive.metastore.properties":
                    (f"spark.hadoop.hive.metastore.uris        {ms}\nspark.sql.catalogImplementation        hive"
                     if ms else ""),
                "spark.extra.properties": "\n".join(env.get("SPARK_EXTRA_PROPERTIES", "").split(";;"))}

    def start_steps(self, head):
        if not head:
            return []
        mk = ("if [ \"$SPARK_WITH_HDFS\" = true ]; then $RUNTIME_PATH/hadoop/bin/hdfs dfs -mkdir -p "
              "/shared/spark-events /shared/spark-warehouse; else mkdir -p $SPARK_HOME/shared/spark-events; fi")
        return [mk, "$SPARK_HOME/sbin/start-history-server.sh"]

    def get_runnable_command(self, target: str, runtime_options: Optional[List[str]] = None):
        """``cloudtik submit`` of a Spark program (reference spark/utils.py:170-179)."""
        q = '"' + target.replace('"', '\\"') + '"'
        if target.endswith(".scala"):
            return ["spark-shell", "-i", q]
        if target.endswith(".jar") or target.endswith(".py"):
            return ["spark-submit"] + list(runtime_options or []) + [q]
        return None
