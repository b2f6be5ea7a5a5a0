"""CLI / executor additions: secrets masked in printed commands and errors (reference
command_executor.py:23-70), `cloudtik run` built-in script resolution, runtime command
groups and the head command set (reference head_scripts.py:70-1054)."""
import pytest
from click.testing import CliRunner


def test_privacy_keys_masked_in_errors():
    from cloudtik_amd.core.executor import (LocalCommandExecutor, ProcessRunnerError, is_key_with_privacy,
                                            with_environment_variables)
    assert is_key_with_privacy("MYSQL_ROOT_PASSWORD") and is_key_with_privacy("AWS_SECRET_ACCESS_KEY")
    assert is_key_with_privacy("api_token") and not is_key_with_privacy("SPARK_EXECUTOR_CORES")
    env = {"DB_PASSWORD": "s3cret-value", "MODE": "x"}
    assert "s3cret-value" not in with_environment_variables("true", env, for_print=True)
    assert "s3cret-value" in with_environment_variables("true", env)
    import subprocess
    ex = LocalCommandExecutor(None, "", {}, "c", subprocess)
    with pytest.raises(ProcessRunnerError) as ei:
        ex.run("[ ${#DB_PASSWORD} -gt 3 ] && exit 7", environment_variables=env)
    msg = str(ei.value)
    assert "s3cret-value" not in msg and "<hidden>" in msg and "code=7" in msg


def test_builtin_script_resolution():
    from cloudtik_amd.core.cluster_operator import _builtin_script_command
    from cloudtik_amd.core.script_registry import registry
    alias = next(iter(registry()))
    assert _builtin_script_command(alias, ["--x", "a b"]).endswith(f"-m {registry()[alias]} --x 'a b'")
    with pytest.raises(ValueError, match="not a built-in script"):
        _builtin_script_command("my_own.py", [])


def test_runtime_command_groups_and_head_commands():
    from cloudtik_amd.cli.main import cli
    for grp in ("ai", "spark", "run"):
        assert grp in cli.commands, grp
    r = CliRunner().invoke(cli, ["head", "--help"])
    assert r.exit_code == 0
    for c in ("attach", "run", "upload", "download", "monitor", "logs", "kill-node", "wait-for-ready",
              "process-status", "cluster-dump", "runtime", "debug-status", "resource-metrics"):
        assert c in r.output, c
    r = CliRunner().invoke(cli, ["head", "runtime", "--help"])
    assert "start" in r.output and "stop" in r.output
    r = CliRunner().invoke(cli, ["spark", "--help"])
    assert "applications" in r.output


def test_head_commands_need_bootstrap_config(tmp_path, monkeypatch):
    from cloudtik_amd.cli.main import cli
    monkeypatch.setenv("HOME", str(tmp_path))
    r = CliRunner().invoke(cli, ["head", "process-status"])
    assert r.exit_code != 0 and "not a head node" in r.output
