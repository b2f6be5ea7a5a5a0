"""Cloud object storage for the Hadoop client configuration (core-site.xml).

What the reference does with ``hadoop-cloud-credential.sh`` (sed over per-cloud core-site
templates plus ``hadoop credential create`` calls) and with its Hadoop source patches
(``source/runtime/hadoop/hadoop-3.3.1/0001`` Azure workload identity and
``0002`` Aliyun ECS RAM role credentials provider), this module does as two pure
functions over the node environment:

* ``export_cloud_storage_env(provider_config)`` -- the provider's ``storage`` section
  (``aws_s3_storage`` / ``gcp_cloud_storage`` / ``azure_cloud_storage`` /
  ``aliyun_oss_storage`` / ``huaweicloud_obs_storage``, reference
  providers/_private/{aws,gcp,_azure,aliyun,huaweicloud}/utils.py ``export_*_storage_config``)
  into the runtime environment (``AWS_CLOUD_STORAGE``, ``AWS_S3_BUCKET`` ...);
* ``cloud_storage_conf(env)`` -> ``(properties, secrets)``: the connector properties that
  go into core-site.xml in clear, and the secret ones (keys, tenant / client ids, token
  file paths) that go into a JCEKS credential store referenced by
  ``hadoop.security.credential.provider.path`` -- never into the XML.

Identity without keys: AWS instance profile, or web identity on EKS (``AWS_WEB_IDENTITY``);
Azure managed identity, or workload identity on AKS (``AZURE_WORKLOAD_IDENTITY``: the
projected ``AZURE_TENANT_ID`` / ``AZURE_CLIENT_ID`` / ``AZURE_FEDERATED_TOKEN_FILE`` feed
``WorkloadIdentityTokenProvider``, the class patch 0001 adds); Aliyun ECS RAM role
(``ALIYUN_ECS_RAM_ROLE_NAME`` feeds ``AliyunEcsRamRoleCredentialsProvider``, patch 0002);
Huawei Cloud ECS agency (``EcsObsCredentialsProvider``). The two patched classes need a
Hadoop build that carries them (the reference's patched 3.3.1 or an upstream release that
merged them); the HDFS fuse / NFS fixes (patches 0003 / 0004) are C and Java changes inside
Hadoop itself and are not carried here.
"""
from __future__ import annotations

import shlex
from typing import Any, Dict, List, Tuple

_ABFS_OAUTH = "org.apache.hadoop.fs.azurebfs.oauth2."
CREDENTIAL_STORE = "credential.jceks"


def _truthy(v) -> bool:
    return str(v).lower() in ("1", "true", "yes")


def export_cloud_storage_env(provider_config: Dict[str, Any]) -> Dict[str, str]:
    """Provider ``storage`` section -> runtime environment (one cloud storage at most).

    On a managed Kubernetes (``provider.cloud_provider``, reference _kubernetes/config.py:1472)
    the storage section is the cloud provider's, and pods authenticate with the cluster's
    federated identity: EKS web identity (``AWS_WEB_IDENTITY``, aws_eks/config.py:879) or
    AKS workload identity (``AZURE_WORKLOAD_IDENTITY``, azure_aks/config.py:1226)."""
    provider_config = provider_config or {}
    env: Dict[str, str] = {}
    cloud = provider_config.get("cloud_provider") or {}
    if provider_config.get("type") == "kubernetes" and cloud:
        if cloud.get("type") == "aws":
            env["AWS_WEB_IDENTITY"] = "true"
        elif cloud.get("type") == "azure":
            env["AZURE_WORKLOAD_IDENTITY"] = "true"
        provider_config = cloud
    storage = provider_config.get("storage") or {}

    def put(name, section, key):
        v = section.get(key)
        if v:
            env[name] = str(v)

    if "aws_s3_storage" in storage:
        s = storage["aws_s3_storage"] or {}
        env["AWS_CLOUD_STORAGE"] = "true"
        put("AWS_S3_BUCKET", s, "s3.bucket")
        put("AWS_S3_ACCESS_KEY_ID", s, "s3.access.key.id")
        put("AWS_S3_SECRET_ACCESS_KEY", s, "s3.secret.access.key")
    elif "gcp_cloud_storage" in storage:
        s = storage["gcp_cloud_storage"] or {}
        env["GCP_CLOUD_STORAGE"] = "true"
        put("GCP_PROJECT_ID", s, "project_id")
        put("GCP_GCS_BUCKET", s, "gcs.bucket")
        put("GCP_GCS_SERVICE_ACCOUNT_CLIENT_EMAIL", s, "gcs.service.account.client.email")
        put("GCP_GCS_SERVICE_ACCOUNT_PRIVATE_KEY_ID", s, "gcs.service.account.private.key.id")
        put("GCP_GCS_SERVICE_ACCOUNT_PRIVATE_KEY", s, "gcs.service.account.private.key")
    elif "azure_cloud_storage" in storage:
        s = storage["azure_cloud_storage"] or {}
        env["AZURE_CLOUD_STORAGE"] = "true"
        put("AZURE_STORAGE_TYPE", s, "azure.storage.type")
        put("AZURE_STORAGE_ACCOUNT", s, "azure.storage.account")
        put("AZURE_CONTAINER", s, "azure.container")
        put("AZURE_ACCOUNT_KEY", s, "azure.account.key")
        mi = provider_config.get("managed_identity_client_id") or s.get("managed.identity.client.id")
        if mi:
            env["AZURE_MANAGED_IDENTITY_CLIENT_ID"] = str(mi)
        if provider_config.get("tenant_id"):
            env["AZURE_MANAGED_IDENTITY_TENANT_ID"] = str(provider_config["tenant_id"])
    elif "aliyun_oss_storage" in storage:
        s = storage["aliyun_oss_storage"] or {}
        env["ALIYUN_CLOUD_STORAGE"] = "true"
        put("ALIYUN_OSS_BUCKET", s, "oss.bucket")
        put("ALIYUN_OSS_INTERNAL_ENDPOINT", s, "oss.internal.endpoint")
        put("ALIYUN_OSS_ACCESS_KEY_ID", s, "oss.access.key.id")
        put("ALIYUN_OSS_ACCESS_KEY_SECRET", s, "oss.access.key.secret")
        if not env.get("ALIYUN_OSS_INTERNAL_ENDPOINT") and provider_config.get("region"):
            env["ALIYUN_OSS_INTERNAL_ENDPOINT"] = f"oss-{provider_config['region']}-internal.aliyuncs.com"
    elif "huaweicloud_obs_storage" in storage:
        s = storage["huaweicloud_obs_storage"] or {}
        env["HUAWEICLOUD_CLOUD_STORAGE"] = "true"
        put("HUAWEICLOUD_OBS_BUCKET", s, "obs.bucket")
        put("HUAWEICLOUD_OBS_ACCESS_KEY", s, "obs.access.key")
        put("HUAWEICLOUD_OBS_SECRET_KEY", s, "obs.secret.key")
        region = provider_config.get("region")
        env["HUAWEICLOUD_OBS_ENDPOINT"] = f"obs.{region}.myhuaweicloud.com" if region else "obs.myhuaweicloud.com"
    return env


def cloud_storage_kind(env: Dict[str, Any]) -> str:
    for kind, flag in (("aws", "AWS_CLOUD_STORAGE"), ("azure", "AZURE_CLOUD_STORAGE"),
                       ("gcp", "GCP_CLOUD_STORAGE"), ("aliyun", "ALIYUN_CLOUD_STORAGE"),
                       ("huaweicloud", "HUAWEICLOUD_CLOUD_STORAGE")):
        if _truthy(env.get(flag, "")):
            return kind
    return "none"


def cloud_storage_uri(env: Dict[str, Any]) -> str:
    """The bucket / container as a Hadoop file system URI ('' when none is configured)."""
    kind = cloud_storage_kind(env)
    if kind == "aws" and env.get("AWS_S3_BUCKET"):
        return f"s3a://{env['AWS_S3_BUCKET']}"
    if kind == "gcp" and env.get("GCP_GCS_BUCKET"):
        return f"gs://{env['GCP_GCS_BUCKET']}"
    if kind == "azure" and env.get("AZURE_CONTAINER") and env.get("AZURE_STORAGE_ACCOUNT"):
        if env.get("AZURE_STORAGE_TYPE") == "blob":
            return f"wasbs://{env['AZURE_CONTAINER']}@{env['AZURE_STORAGE_ACCOUNT']}.blob.core.windows.net"
        return f"abfs://{env['AZURE_CONTAINER']}@{env['AZURE_STORAGE_ACCOUNT']}.dfs.core.windows.net"
    if kind == "aliyun" and env.get("ALIYUN_OSS_BUCKET"):
        return f"oss://{env['ALIYUN_OSS_BUCKET']}"
    if kind == "huaweicloud" and env.get("HUAWEICLOUD_OBS_BUCKET"):
        return f"obs://{env['HUAWEICLOUD_OBS_BUCKET']}"
    return ""


def cloud_storage_conf(env: Dict[str, Any]) -> Tuple[Dict[str, str], Dict[str, str]]:
    """(core-site properties, credential-store secrets) for the node's cloud storage."""
    props, secrets, _ = _storage_conf(env)
    return props, secrets


def cloud_storage_secret_vars(env: Dict[str, Any]) -> Dict[str, str]:
    """credential-store alias -> NAME of the node environment variable holding its value
    (the configure steps reference the variable, never the secret itself)."""
    return _storage_conf(env)[2]


def _storage_conf(env: Dict[str, Any]) -> Tuple[Dict[str, str], Dict[str, str], Dict[str, str]]:
    kind = cloud_storage_kind(env)
    props: Dict[str, str] = {}
    secrets: Dict[str, str] = {}
    sources: Dict[str, str] = {}

    def secret(name, var):
        if env.get(var):
            secrets[name] = str(env[var])
            sources[name] = var

    if kind == "aws":
        if env.get("AWS_S3_ACCESS_KEY_ID"):
            props["fs.s3a.aws.credentials.provider"] = "org.apache.hadoop.fs.s3a.SimpleAWSCredentialsProvider"
            props["fs.s3a.access.key"] = str(env["AWS_S3_ACCESS_KEY_ID"])
            secret("fs.s3a.secret.key", "AWS_S3_SECRET_ACCESS_KEY")
        elif _truthy(env.get("AWS_WEB_IDENTITY", "")):
            props["fs.s3a.aws.credentials.provider"] = "com.amazonaws.auth.WebIdentityTokenCredentialsProvider"
        else:
            props["fs.s3a.aws.credentials.provider"] = "com.amazonaws.auth.InstanceProfileCredentialsProvider"
    elif kind == "gcp":
        props["fs.gs.impl"] = "com.google.cloud.hadoop.fs.gcs.GoogleHadoopFileSystem"
        props["fs.AbstractFileSystem.gs.impl"] = "com.google.cloud.hadoop.fs.gcs.GoogleHadoopFS"
        if env.get("GCP_PROJECT_ID"):
            props["fs.gs.project.id"] = str(env["GCP_PROJECT_ID"])
        if env.get("GCP_GCS_SERVICE_ACCOUNT_CLIENT_EMAIL"):
            props["fs.gs.auth.service.account.enable"] = "true"
            props["fs.gs.auth.service.account.email"] = str(env["GCP_GCS_SERVICE_ACCOUNT_CLIENT_EMAIL"])
            props["fs.gs.auth.service.account.private.key.id"] = str(
                env.get("GCP_GCS_SERVICE_ACCOUNT_PRIVATE_KEY_ID", ""))
            secret("fs.gs.auth.service.account.private.key", "GCP_GCS_SERVICE_ACCOUNT_PRIVATE_KEY")
    elif kind == "azure":
        account = env.get("AZURE_STORAGE_ACCOUNT", "")
        endpoint = "blob" if env.get("AZURE_STORAGE_TYPE") == "blob" else "dfs"
        if env.get("AZURE_ACCOUNT_KEY"):
            if endpoint == "dfs":
                props["fs.azure.account.auth.type"] = "SharedKey"
            secret(f"fs.azure.account.key.{account}.{endpoint}.core.windows.net", "AZURE_ACCOUNT_KEY")
        elif endpoint == "dfs":
            props["fs.azure.account.auth.type"] = "OAuth"
            workload = _truthy(env.get("AZURE_WORKLOAD_IDENTITY", ""))
            props["fs.azure.account.oauth.provider.type"] = _ABFS_OAUTH + (
                "WorkloadIdentityTokenProvider" if workload else "MsiTokenProvider")
            tenant, client = env.get("AZURE_MANAGED_IDENTITY_TENANT_ID"), env.get("AZURE_MANAGED_IDENTITY_CLIENT_ID")
            tenant_var, client_var = "AZURE_MANAGED_IDENTITY_TENANT_ID", "AZURE_MANAGED_IDENTITY_CLIENT_ID"
            if workload:
                # the pod's projected identity (AKS workload identity webhook) wins
                if env.get("AZURE_TENANT_ID"):
                    tenant_var = "AZURE_TENANT_ID"
                if env.get("AZURE_CLIENT_ID"):
                    client_var = "AZURE_CLIENT_ID"
                secret("fs.azure.account.oauth2.msi.authority", "AZURE_AUTHORITY_HOST")
                secret("fs.azure.account.oauth2.token.file", "AZURE_FEDERATED_TOKEN_FILE")
            secret("fs.azure.account.oauth2.msi.tenant", tenant_var)
            secret("fs.azure.account.oauth2.client.id", client_var)
    elif kind == "aliyun":
        props["fs.oss.impl"] = "org.apache.hadoop.fs.aliyun.oss.AliyunOSSFileSystem"
        if env.get("ALIYUN_OSS_INTERNAL_ENDPOINT"):
            props["fs.oss.endpoint"] = str(env["ALIYUN_OSS_INTERNAL_ENDPOINT"])
        if not (env.get("ALIYUN_OSS_ACCESS_KEY_ID") and env.get("ALIYUN_OSS_ACCESS_KEY_SECRET")):
            props["fs.oss.credentials.provider"] = "org.apache.hadoop.fs.aliyun.oss.AliyunEcsRamRoleCredentialsProvider"
        secret("fs.oss.accessKeyId", "ALIYUN_OSS_ACCESS_KEY_ID")
        secret("fs.oss.accessKeySecret", "ALIYUN_OSS_ACCESS_KEY_SECRET")
        secret("fs.oss.ecs.ramRoleName", "ALIYUN_ECS_RAM_ROLE_NAME")
    elif kind == "huaweicloud":
        props["fs.obs.impl"] = "org.apache.hadoop.fs.obs.OBSFileSystem"
        props["fs.AbstractFileSystem.obs.impl"] = "org.apache.hadoop.fs.obs.OBS"
        if env.get("HUAWEICLOUD_OBS_ENDPOINT"):
            props["fs.obs.endpoint"] = str(env["HUAWEICLOUD_OBS_ENDPOINT"])
        if not (env.get("HUAWEICLOUD_OBS_ACCESS_KEY") and env.get("HUAWEICLOUD_OBS_SECRET_KEY")):
            props["fs.obs.security.provider"] = "com.obs.services.EcsObsCredentialsProvider"
        secret("fs.obs.access.key", "HUAWEICLOUD_OBS_ACCESS_KEY")
        secret("fs.obs.secret.key", "HUAWEICLOUD_OBS_SECRET_KEY")
    return props, secrets, sources


def properties_xml(props: Dict[str, str], credential_file: str = "") -> str:
    from xml.sax.saxutils import escape
    items = dict(props)
    if credential_file:
        items["hadoop.security.credential.provider.path"] = f"jceks://file@{credential_file}"
    return "\n".join(f"  <property><name>{escape(k)}</name><value>{escape(str(v))}</value></property>"
                     for k, v in items.items())


def credential_commands(secret_vars: Dict[str, str], hadoop_home: str, credential_file: str) -> List[str]:
    """``hadoop credential create`` per secret into a fresh store (rewritten every configure).

    ``secret_vars`` maps each alias to the NAME of the environment variable that holds it; the
    commands expand ``"$VAR"`` when they run (the steps run with the node environment), so no
    secret value appears in a step string, a failed step's error message or a log."""
    if not secret_vars:
        return []
    store = f"jceks://file@{credential_file}"
    cmds = [f"rm -f {shlex.quote(credential_file)}"]
    for name, var in secret_vars.items():
        if not var.replace("_", "").isalnum():
            raise ValueError(f"not an environment variable name: {var!r}")
        cmds.append(f"{shlex.quote(hadoop_home + '/bin/hadoop')} credential create {shlex.quote(name)} "
                    f"-value \"${var}\" -provider {shlex.quote(store)} > /dev/null")
    return cmds
