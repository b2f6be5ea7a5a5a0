"""Replication bootstrap of the database runtimes: the commands each node role runs after (or,
for a Postgres standby, before) its server starts, so that a cluster with
``cluster_mode: replication`` (or ``group_replication`` / ``sharding``) really replicates
instead of running N independent servers.

Reference behaviour (what, not how):

* MySQL -- runtime/mysql/scripts/mysql-init.sh + mysql.sh:340-402: a replication user on
  every node (binlog off for that statement), ``CHANGE REPLICATION SOURCE TO`` the head with
  GTID auto-positioning on the replicas; for group replication the recovery channel
  credentials, the head bootstrapping the group (``group_replication_bootstrap_group``) and the
  others ``START GROUP_REPLICATION``.
* PostgreSQL -- runtime/postgres/scripts/postgres.sh:515-533, repmgr.sh, repmgr-init.sh: a
  replication role on the primary; a standby is (re)built from the primary with a base backup
  (``standby.signal`` + ``primary_conninfo``) instead of initialising its own cluster; with
  repmgr, ``primary register`` / ``standby clone`` + ``standby register`` and ``repmgrd`` for
  automatic failover.
* MongoDB -- runtime/mongodb/scripts/mongodb.sh:600-680, mongodb-sharding.sh: the head
  initiates the replica set with itself (priority 5), members are added from the primary;
  sharded: a config-server replica set + ``mongos`` on the head, the workers grouped into
  shard replica sets whose first member initiates its set and registers it with
  ``sh.addShard``.

Every step is idempotent on re-run (a marker file, ``IF NOT EXISTS``, "already initialized"
tolerated) and waits for the peer it needs with a bounded retry loop, because the head and the
workers start in no particular order.  The steps are plain bash lines run by
``RuntimeBase._run_steps`` -- tests capture them per node role (tests/test_replication.py).
"""
from __future__ import annotations

import shlex
import uuid
from typing import Any, Dict, List, Optional, Tuple

REPL_USER = "repl_user"
DEFAULT_PASSWORD = "cloudtik"


def retry(cmd: str, tries: int = 60, delay: float = 2) -> str:
    """bash: run ``cmd`` until it succeeds, at most ``tries`` times; fails after that.  One
    brace group, so ``a && retry(b) && c`` chains as written."""
    return (f"{{ _ok=0; for _i in $(seq {tries}); do if ( {cmd} ); then _ok=1; break; fi; sleep {delay}; done; "
            f"[ $_ok -eq 1 ]; }}")


def once(marker: str, cmd: str) -> str:
    """bash: run ``cmd`` unless ``marker`` exists; create the marker when it succeeded."""
    return f"[ -f {marker} ] || {{ {cmd} && touch {marker}; }}"


def feed_stdin(prefix: str, body: str) -> str:
    """bash: ``printf '%s\\n' '<body>' | prefix`` -- the body (SQL) on the command's stdin, single-
    quoted so nothing in it is expanded.  One shell word, so the step composes with ``&&`` / ``;``
    / ``( )`` anywhere on a line (a here-document would end only at a line holding its bare tag,
    swallowing whatever the caller appends after it)."""
    return f"printf '%s\\n' {shlex.quote(body.rstrip())} | {prefix}"


def _sq(v: str) -> str:
    """SQL single-quoted literal."""
    return "'" + str(v).replace("'", "''") + "'"


# ------------------------------------------------------------------------------- MySQL
def mysql_group_name(cluster: str) -> str:
    """Group replication needs one UUID shared by the members: derived from the cluster name."""
    return str(uuid.uuid5(uuid.NAMESPACE_DNS, f"cloudtik-mysql-{cluster}"))


def mysql_group_conf(c: Dict[str, Any], port: int) -> List[str]:
    """my.cnf lines of a group-replication member (single primary unless multi_primary)."""
    gport = int(c["cfg"].get("group_replication_port", 33061))
    seeds = [c["head_ip"]] + [ip for _, ip in c["members"] if ip != c["head_ip"]]
    multi = bool(c["cfg"].get("multi_primary"))
    return ["plugin_load_add = group_replication.so",
            f"group_replication_group_name = {mysql_group_name(c['cluster'])}",
            "group_replication_start_on_boot = OFF",
            "group_replication_bootstrap_group = OFF",
            f"group_replication_local_address = {c['ip']}:{gport}",
            f"group_replication_group_seeds = {','.join(f'{ip}:{gport}' for ip in seeds)}",
            f"group_replication_single_primary_mode = {'OFF' if multi else 'ON'}",
            f"group_replication_enforce_update_everywhere_checks = {'ON' if multi else 'OFF'}",
            "disabled_storage_engines = \"MyISAM,BLACKHOLE,FEDERATED,ARCHIVE,MEMORY\""]


def mysql_sql(body: str) -> str:
    return feed_stdin("sudo mysql -uroot --protocol=socket", body)


def mysql_bootstrap_steps(c: Dict[str, Any]) -> List[str]:
    """Steps after mysqld started on this node, by role and cluster mode."""
    cfg = c["cfg"]
    mode = cfg.get("cluster_mode", "none")
    if mode not in ("replication", "group_replication"):
        return []
    pw = cfg.get("replication_password", DEFAULT_PASSWORD)
    port = int(cfg.get("port", 3306))
    marker = f"{c['dir']}/.replication-initialized"
    grants = [f"GRANT REPLICATION SLAVE ON *.* TO '{REPL_USER}'@'%';"]
    if mode == "group_replication":
        grants += [f"GRANT {g} ON *.* TO '{REPL_USER}'@'%';"
                   for g in ("CONNECTION_ADMIN", "BACKUP_ADMIN", "GROUP_REPLICATION_STREAM")]
    # the replication user is created on EVERY node with the binlog off for the statements:
    # it must not replicate (a replica would then try to create it twice)
    user_sql = "\n".join(["SET SESSION sql_log_bin = 0;",
                          f"CREATE USER IF NOT EXISTS '{REPL_USER}'@'%' IDENTIFIED BY {_sq(pw)};"] + grants +
                         ["FLUSH PRIVILEGES;", "SET SESSION sql_log_bin = 1;"])
    wait_local = retry("sudo mysqladmin -uroot --protocol=socket ping >/dev/null 2>&1", tries=60, delay=1)
    steps = [wait_local]
    if mode == "replication":
        if c["head"]:
            steps.append(once(marker, mysql_sql(user_sql)))
        else:
            src = "\n".join([f"CHANGE REPLICATION SOURCE TO SOURCE_HOST = {_sq(c['head_ip'])}, SOURCE_PORT = {port},",
                             f"  SOURCE_USER = '{REPL_USER}', SOURCE_PASSWORD = {_sq(pw)},",
                             "  SOURCE_AUTO_POSITION = 1, GET_SOURCE_PUBLIC_KEY = 1;",
                             "START REPLICA;"])
            # the source must accept the replication user before the replica connects
            probe = (f"mysqladmin -h {c['head_ip']} -P {port} -u{REPL_USER} -p{shlex.quote(pw)} "
                     f"ping >/dev/null 2>&1")
            steps.append(once(marker, f"{mysql_sql(user_sql)} && {retry(probe)} && {mysql_sql(src)}"))
        return steps
    # group replication
    recovery = (f"CHANGE REPLICATION SOURCE TO SOURCE_USER = '{REPL_USER}', SOURCE_PASSWORD = {_sq(pw)} "
                "FOR CHANNEL 'group_replication_recovery';")
    on_boot = (f"printf '[mysqld]\\ngroup_replication_start_on_boot = ON\\n' | "
               f"sudo tee /etc/mysql/mysql.conf.d/zz-cloudtik-gr-boot.cnf >/dev/null 2>&1 || true")
    if c["head"]:
        boot = "\n".join(["SET GLOBAL group_replication_bootstrap_group = ON;", "START GROUP_REPLICATION;",
                          "SET GLOBAL group_replication_bootstrap_group = OFF;"])
        steps.append(once(marker, f"{mysql_sql(user_sql + chr(10) + recovery)} && {mysql_sql(boot)} && {on_boot}"))
    else:
        # joins through the seeds (the head bootstrapped the group): retried until the group exists
        join = retry(mysql_sql("START GROUP_REPLICATION;"), tries=60, delay=3)
        steps.append(once(marker, f"{mysql_sql(user_sql + chr(10) + recovery)} && {join} && {on_boot}"))
    return steps


# ------------------------------------------------------------------------------- PostgreSQL
PG_DATA = "$(ls -d /var/lib/postgresql/*/main 2>/dev/null | head -1)"


def psql(body: str, host: Optional[str] = None, extra: str = "") -> str:
    h = f" -h {host}" if host else ""
    return feed_stdin(f"sudo -u postgres psql -v ON_ERROR_STOP=1{h}{extra}", body)


def repmgr_conf(c: Dict[str, Any], data_dir: str) -> str:
    """repmgr.conf of this node (node ids: head 1, worker seq + 1, unique and stable)."""
    cfg = c["cfg"]
    rp = cfg.get("repmgr") or {}
    node_id = 1 if c["head"] else int(c["seq"]) + 1
    conf_path = f"{c['dir']}/repmgr.conf"
    lines = [f"node_id={node_id}", f"node_name='{c['cluster']}-{node_id}'",
             f"conninfo='host={c['ip']} port={int(cfg.get('port', 5432))} user=repmgr dbname=repmgr connect_timeout=5'",
             f"data_directory='{data_dir}'", "use_replication_slots=yes",
             f"failover='{'automatic' if rp.get('failover', 'automatic') == 'automatic' else 'manual'}'",
             f"promote_command='repmgr standby promote -f {conf_path} --log-to-file'",
             f"follow_command='repmgr standby follow -f {conf_path} --log-to-file --upstream-node-id=%n'",
             "monitoring_history=yes", f"reconnect_attempts={int(rp.get('reconnect_attempts', 6))}",
             f"reconnect_interval={int(rp.get('reconnect_interval', 10))}",
             f"log_file='{c['dir']}/logs/repmgrd.log'", "service_start_command='sudo service postgresql start'",
             "service_stop_command='sudo service postgresql stop'"]
    return "\n".join(lines) + "\n"


def postgres_repmgr_enabled(cfg: Dict[str, Any]) -> bool:
    return cfg.get("cluster_mode", "none") == "replication" and bool((cfg.get("repmgr") or {}).get("enabled"))


def postgres_pre_start_steps(c: Dict[str, Any]) -> List[str]:
    """A standby is built from the primary BEFORE its server starts: its data directory is
    replaced by a base backup of the primary (pg_basebackup -R writes standby.signal and
    primary_conninfo; repmgr ``standby clone`` does the same through repmgr).  Skipped once the
    data directory already is a standby."""
    cfg = c["cfg"]
    if cfg.get("cluster_mode", "none") != "replication" or c["head"]:
        return []
    pw = cfg.get("replication_password", DEFAULT_PASSWORD)
    port = int(cfg.get("port", 5432))
    user = cfg.get("replication_user", REPL_USER)
    primary_up = f"pg_isready -h {c['head_ip']} -p {port} -q"
    if postgres_repmgr_enabled(cfg):
        clone = (f"sudo -u postgres env PGPASSWORD={shlex.quote(cfg.get('repmgr_password', pw))} "
                 f"repmgr -h {c['head_ip']} -p {port} -U repmgr -d repmgr -f {c['dir']}/repmgr.conf "
                 "standby clone --force")
    else:
        clone = (f"sudo -u postgres env PGPASSWORD={shlex.quote(pw)} pg_basebackup -h {c['head_ip']} -p {port} "
                 f"-U {user} -D \"$D\" -X stream -R")
    return [f"D={PG_DATA}; [ -n \"$D\" ] || exit 1; [ -f \"$D/standby.signal\" ] || {{ "
            f"{retry(primary_up, tries=90, delay=2)} || exit 1; sudo service postgresql stop; "
            f"sudo rm -rf \"$D.cloudtik-old\" && sudo mv \"$D\" \"$D.cloudtik-old\" && "
            f"sudo install -d -o postgres -g postgres -m 700 \"$D\" && {clone} && "
            f"sudo chown -R postgres:postgres \"$D\"; }}"]


def postgres_bootstrap_steps(c: Dict[str, Any]) -> List[str]:
    """Steps after the server started: the primary's replication (and repmgr) roles, repmgr
    registration and its daemon on every node."""
    cfg = c["cfg"]
    if cfg.get("cluster_mode", "none") != "replication":
        return []
    pw = cfg.get("replication_password", DEFAULT_PASSWORD)
    user = cfg.get("replication_user", REPL_USER)
    marker = f"{c['dir']}/.replication-initialized"
    wait_local = retry("pg_isready -q", tries=60, delay=1)
    steps = [wait_local]
    repmgr = postgres_repmgr_enabled(cfg)
    conf = f"{c['dir']}/repmgr.conf"
    if c["head"]:
        sql = ["DO $$ BEGIN",
               f"  IF NOT EXISTS (SELECT FROM pg_roles WHERE rolname = {_sq(user)}) THEN",
               f"    CREATE ROLE {user} WITH REPLICATION LOGIN PASSWORD {_sq(pw)};",
               "  END IF;"]
        if repmgr:
            rpw = cfg.get("repmgr_password", pw)
            sql += ["  IF NOT EXISTS (SELECT FROM pg_roles WHERE rolname = 'repmgr') THEN",
                    f"    CREATE ROLE repmgr WITH SUPERUSER REPLICATION LOGIN PASSWORD {_sq(rpw)};",
                    "  END IF;"]
        sql.append("END $$;")
        cmd = psql("\n".join(sql))
        if repmgr:
            cmd += (" && (sudo -u postgres psql -tAc \"SELECT 1 FROM pg_database WHERE datname='repmgr'\" | "
                    "grep -q 1 || sudo -u postgres createdb -O repmgr repmgr)"
                    f" && sudo -u postgres repmgr -f {conf} primary register --force")
        steps.append(once(marker, cmd))
    elif repmgr:
        steps.append(once(marker, f"sudo -u postgres repmgr -f {conf} standby register --force"))
    if repmgr:
        steps.append(f"pgrep -f 'repmgrd -f {conf}' >/dev/null || sudo -u postgres repmgrd -f {conf} --daemonize")
    return steps


# ------------------------------------------------------------------------------- MongoDB
def mongo_eval(js: str, host: str = "127.0.0.1", port: int = 27017) -> str:
    return f"mongosh --quiet --host {host} --port {port} --eval {shlex.quote(js)}"


def mongo_shard_layout(members: List[Tuple[int, str]], shard_size: int, cluster: str) -> List[Dict[str, Any]]:
    """Workers (sequence order) grouped into shard replica sets of ``shard_size`` members."""
    size = max(1, int(shard_size))
    out = []
    for k in range(0, len(members), size):
        grp = members[k:k + size]
        out.append({"name": f"{cluster}-shard{k // size}", "members": [ip for _, ip in grp]})
    return out


def mongo_initiate(rs: str, host_port: str, priority: int = 5, configsvr: bool = False) -> str:
    cs = ", configsvr: true" if configsvr else ""
    return ("try { rs.initiate({_id: %s%s, members: [{_id: 0, host: %s, priority: %d}]}) } "
            'catch (e) { if (e.codeName !== "AlreadyInitialized") throw e }'
            % (_js(rs), cs, _js(host_port), priority))


def mongo_add(host_port: str) -> str:
    """Run on the primary: add a member unless it is one already (reconfig is refused while
    the set has no primary: the caller retries)."""
    return ('if (!rs.isMaster().ismaster) throw new Error("not primary"); '
            "if (!rs.conf().members.some(m => m.host === %s)) { const r = rs.add({host: %s}); "
            "if (r.ok !== 1) throw new Error(JSON.stringify(r)) }" % (_js(host_port), _js(host_port)))


def _js(s: str) -> str:
    """A JavaScript string literal in double quotes (the whole script is then single-quoted
    for the shell without any quote juggling)."""
    import json
    return json.dumps(str(s))


def mongodb_bootstrap_steps(c: Dict[str, Any]) -> List[str]:
    cfg = c["cfg"]
    mode = cfg.get("cluster_mode", "none")
    port = int(cfg.get("port", 27017))
    if mode == "replication":
        rs = cfg.get("replication_set_name") or f"{c['cluster']}-rs"
        local_up = retry(mongo_eval("db.adminCommand({ping: 1})", port=port), tries=60, delay=1)
        if c["head"]:
            return [local_up, retry(mongo_eval(mongo_initiate(rs, f"{c['head_ip']}:{port}"), port=port), tries=30)]
        return [local_up, retry(mongo_eval(mongo_add(f"{c['ip']}:{port}"), host=c["head_ip"], port=port),
                                tries=90, delay=2)]
    if mode != "sharding":
        return []
    cfg_port = int(cfg.get("config_server_port", 27019))
    shard_port = int(cfg.get("shard_server_port", 27018))
    if c["head"]:
        cfg_rs = f"{c['cluster']}-cfg"
        return [retry(mongo_eval("db.adminCommand({ping: 1})", port=cfg_port), tries=60, delay=1),
                retry(mongo_eval(mongo_initiate(cfg_rs, f"{c['head_ip']}:{cfg_port}", configsvr=True),
                                 port=cfg_port), tries=30),
                f"pgrep -f 'mongos --config {c['dir']}/mongos.conf' >/dev/null || mongos --config {c['dir']}/mongos.conf"]
    # worker: which shard replica set this node belongs to, and whether it is its first member
    layout = mongo_shard_layout(c["members"], cfg.get("shard_size", 1), c["cluster"])
    mine = next((s for s in layout if c["ip"] in s["members"]), None)
    if mine is None:
        return []
    first = mine["members"][0]
    steps = [retry(mongo_eval("db.adminCommand({ping: 1})", port=shard_port), tries=60, delay=1)]
    if c["ip"] == first:
        steps.append(retry(mongo_eval(mongo_initiate(mine["name"], f"{first}:{shard_port}"), port=shard_port),
                           tries=30))
        hosts = ",".join(f"{ip}:{shard_port}" for ip in mine["members"])
        add_shard = ("const s = db.adminCommand({listShards: 1}).shards || []; "
                     "if (!s.some(x => x._id === %s)) { const r = sh.addShard(%s); "
                     "if (r.ok !== 1) throw new Error(JSON.stringify(r)) }"
                     % (_js(mine["name"]), _js(f"{mine['name']}/{hosts.split(',')[0]}")))
        steps.append(retry(mongo_eval(add_shard, host=c["head_ip"], port=port), tries=90, delay=2))
    else:
        steps.append(retry(mongo_eval(mongo_add(f"{c['ip']}:{shard_port}"), host=first, port=shard_port),
                           tries=90, delay=2))
    return steps


# ------------------------------------------------------------------------------- Redis sentinel
def redis_sentinel_conf(c: Dict[str, Any]) -> str:
    """Sentinel monitoring the head (the replication master) with a majority quorum of the
    nodes running a sentinel (reference runtime/redis/scripts/redis-sentinel.sh)."""
    cfg = c["cfg"]
    sc = cfg.get("sentinel") or {}
    port = int(cfg.get("port", 6379))
    name = sc.get("master_name", f"{c['cluster']}-master")
    n = 1 + len(c["members"])
    quorum = int(sc.get("quorum", n // 2 + 1))
    lines = [f"port {int(sc.get('port', 26379))}", "bind 0.0.0.0", "protected-mode no",
             f"dir {c['dir']}/data", f"logfile {c['dir']}/logs/sentinel.log",
             f"sentinel monitor {name} {c['head_ip']} {port} {quorum}",
             f"sentinel down-after-milliseconds {name} {int(sc.get('down_after_ms', 5000))}",
             f"sentinel failover-timeout {name} {int(sc.get('failover_timeout_ms', 60000))}",
             f"sentinel parallel-syncs {name} 1", "sentinel resolve-hostnames yes"]
    if cfg.get("password"):
        lines.append(f"sentinel auth-pass {name} {cfg['password']}")
    return "\n".join(lines) + "\n"
