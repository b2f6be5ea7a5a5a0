"""Instance templates for ``from: <provider>/<size>`` and ``from: <provider>/gpu/<family>/<size>``
(reference python/cloudtik/templates/**, 186 YAML files) generated from compact tables.

A template fixes the head and worker ``node_config`` of the ``head.default`` /
``worker.default`` node types for one provider: the instance type (or Kubernetes pod
resources), the boot disk and, for workers, a data disk.  Instead of shipping one YAML file
per (provider, size, GPU family) combination, the tables below describe

* size classes -- ``small``, ``medium``, ``standard``, ``large``, ``very-large`` with
  ``-highmem`` (memory-optimised family) variants and a ``latest/`` newer generation;
* GPU families per provider -- the NVIDIA families the reference's example configs name
  (t4, v100, a100, ...) so those configs keep loading, and the AMD Instinct instances
  (``gpu/mi300x/...`` on Azure ND MI300X v5; on-premise / local MI355X nodes use
  ``templates/onpremise`` / ``templates/local``) that this framework targets.

User templates (``$CLOUDTIK_USER_TEMPLATES``) and files under ``cloudtik_amd/templates``
take precedence; :func:`synthesize` is only consulted when no file exists.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

PROVIDERS = ("aws", "azure", "gcp", "aliyun", "huaweicloud", "kubernetes")
K8S_CLOUDS = {"eks": "aws", "aks": "azure", "gke": "gcp"}

# size class -> (head vCPU, worker vCPU, worker data disk GB)
SIZES: Dict[str, Tuple[int, int, int]] = {
    "small": (4, 4, 100), "medium": (8, 8, 100), "standard": (8, 8, 200),
    "large": (8, 16, 400), "very-large": (16, 32, 800),
}

# provider -> {vCPU: instance}, for (general, highmem) x (current, latest)
_GENERAL = {
    "aws": ({4: "m5.xlarge", 8: "m5.2xlarge", 16: "m5.4xlarge", 32: "m5.8xlarge"},
            {4: "m6i.xlarge", 8: "m6i.2xlarge", 16: "m6i.4xlarge", 32: "m6i.8xlarge"}),
    "azure": ({4: "Standard_D4s_v4", 8: "Standard_D8s_v4", 16: "Standard_D16s_v4", 32: "Standard_D32s_v4"},
              {4: "Standard_D4s_v5", 8: "Standard_D8s_v5", 16: "Standard_D16s_v5", 32: "Standard_D32s_v5"}),
    "gcp": ({4: "n2-standard-4", 8: "n2-standard-8", 16: "n2-standard-16", 32: "n2-standard-32"},
            {4: "c3-standard-4", 8: "c3-standard-8", 16: "c3-standard-22", 32: "c3-standard-44"}),
    "aliyun": ({4: "ecs.g7.xlarge", 8: "ecs.g7.2xlarge", 16: "ecs.g7.4xlarge", 32: "ecs.g7.8xlarge"},
               {4: "ecs.g8i.xlarge", 8: "ecs.g8i.2xlarge", 16: "ecs.g8i.4xlarge", 32: "ecs.g8i.8xlarge"}),
    "huaweicloud": ({4: "s6.xlarge.2", 8: "s6.2xlarge.2", 16: "s6.4xlarge.2", 32: "s6.8xlarge.2"},
                    {4: "s7.xlarge.2", 8: "s7.2xlarge.2", 16: "s7.4xlarge.2", 32: "s7.8xlarge.2"}),
}
_HIGHMEM = {
    "aws": ({4: "r5.xlarge", 8: "r5.2xlarge", 16: "r5.4xlarge", 32: "r5.8xlarge"},
            {4: "r6i.xlarge", 8: "r6i.2xlarge", 16: "r6i.4xlarge", 32: "r6i.8xlarge"}),
    "azure": ({4: "Standard_E4s_v4", 8: "Standard_E8s_v4", 16: "Standard_E16s_v4", 32: "Standard_E32s_v4"},
              {4: "Standard_E4s_v5", 8: "Standard_E8s_v5", 16: "Standard_E16s_v5", 32: "Standard_E32s_v5"}),
    "gcp": ({4: "n2-highmem-4", 8: "n2-highmem-8", 16: "n2-highmem-16", 32: "n2-highmem-32"},
            {4: "c3-highmem-4", 8: "c3-highmem-8", 16: "c3-highmem-22", 32: "c3-highmem-44"}),
    "aliyun": ({4: "ecs.r7.xlarge", 8: "ecs.r7.2xlarge", 16: "ecs.r7.4xlarge", 32: "ecs.r7.8xlarge"},
               {4: "ecs.r8i.xlarge", 8: "ecs.r8i.2xlarge", 16: "ecs.r8i.4xlarge", 32: "ecs.r8i.8xlarge"}),
    "huaweicloud": ({4: "m6.xlarge.8", 8: "m6.2xlarge.8", 16: "m6.4xlarge.8", 32: "m6.8xlarge.8"},
                    {4: "m7.xlarge.8", 8: "m7.2xlarge.8", 16: "m7.4xlarge.8", 32: "m7.8xlarge.8"}),
}

# provider -> family -> size -> (worker instance or (machine, accelerator, count), GPUs)
_GPU = {
    "aws": {
        "t4": {"very-small": ("g4dn.xlarge", 1), "small": ("g4dn.2xlarge", 1), "standard": ("g4dn.8xlarge", 1),
               "large": ("g4dn.12xlarge", 4), "very-large": ("g4dn.metal", 8)},
        "v100": {"standard": ("p3.2xlarge", 1), "large": ("p3.8xlarge", 4), "very-large": ("p3.16xlarge", 8),
                 "very-large-x": ("p3dn.24xlarge", 8)},
        "a100": {"very-large": ("p4d.24xlarge", 8)},
    },
    "azure": {
        "t4": {"very-small": ("Standard_NC4as_T4_v3", 1), "small": ("Standard_NC8as_T4_v3", 1),
               "standard": ("Standard_NC16as_T4_v3", 1), "large": ("Standard_NC64as_T4_v3", 4)},
        "v100": {"medium": ("Standard_NC6s_v3", 1), "standard": ("Standard_NC12s_v3", 2),
                 "large": ("Standard_NC24s_v3", 4)},
        "a100": {"medium": ("Standard_NC24ads_A100_v4", 1), "standard": ("Standard_NC48ads_A100_v4", 2),
                 "large": ("Standard_NC96ads_A100_v4", 4), "very-large": ("Standard_ND96asr_v4", 8)},
        "mi300x": {"very-large": ("Standard_ND96isr_MI300X_v5", 8)},
    },
    "gcp": {
        "t4": {"very-small": (("n1-standard-4", "nvidia-tesla-t4", 1), 1),
               "small": (("n1-standard-8", "nvidia-tesla-t4", 1), 1),
               "medium": (("n1-standard-8", "nvidia-tesla-t4", 2), 2),
               "standard": (("n1-standard-16", "nvidia-tesla-t4", 1), 1),
               "large": (("n1-standard-32", "nvidia-tesla-t4", 4), 4)},
        "v100": {"medium": (("n1-standard-8", "nvidia-tesla-v100", 1), 1),
                 "standard": (("n1-standard-16", "nvidia-tesla-v100", 2), 2),
                 "large": (("n1-standard-32", "nvidia-tesla-v100", 4), 4),
                 "very-large": (("n1-standard-64", "nvidia-tesla-v100", 8), 8)},
        "a100-40": {"medium": ("a2-highgpu-1g", 1), "standard": ("a2-highgpu-2g", 2), "large": ("a2-highgpu-4g", 4),
                    "very-large": ("a2-highgpu-8g", 8), "utra-large": ("a2-megagpu-16g", 16)},
        "a100-80": {"medium": ("a2-ultragpu-1g", 1), "standard": ("a2-ultragpu-2g", 2),
                    "large": ("a2-ultragpu-4g", 4), "very-large": ("a2-ultragpu-8g", 8)},
    },
    "aliyun": {
        "t4": {"very-small": ("ecs.gn6i-c4g1.xlarge", 1), "small": ("ecs.gn6i-c8g1.2xlarge", 1),
               "medium": ("ecs.gn6i-c16g1.4xlarge", 1), "standard": ("ecs.gn6i-c24g1.6xlarge", 1),
               "large": ("ecs.gn6i-c24g1.12xlarge", 2)},
        "v100-16": {"standard": ("ecs.gn6v-c8g1.2xlarge", 1), "large": ("ecs.gn6v-c8g1.8xlarge", 4),
                    "very-large": ("ecs.gn6v-c8g1.16xlarge", 8), "very-large-x": ("ecs.gn6v-c10g1.20xlarge", 8)},
        "v100-32": {"standard": ("ecs.gn6e-c12g1.3xlarge", 1), "large": ("ecs.gn6e-c12g1.12xlarge", 4),
                    "very-large": ("ecs.gn6e-c12g1.24xlarge", 8)},
        "a100-40": {"standard": ("ecs.gn7-c12g1.3xlarge", 1), "large": ("ecs.gn7-c13g1.13xlarge", 4),
                    "very-large": ("ecs.gn7-c13g1.26xlarge", 8)},
        "a100-80": {"standard": ("ecs.gn7e-c16g1.4xlarge", 1), "large": ("ecs.gn7e-c16g1.16xlarge", 4),
                    "very-large": ("ecs.gn7e-c16g1.32xlarge", 8)},
    },
}


def _disk(provider: str, size_gb: int, data: bool) -> Dict[str, Any]:
    if provider == "aws":
        return {"DeviceName": "/dev/sdf" if data else "/dev/sda1",
                "Ebs": {"VolumeSize": size_gb, "VolumeType": "gp3" if data else "gp2", "DeleteOnTermination": True}}
    raise KeyError(provider)


def _node_config(provider: str, instance, boot_gb: int, data_gb: int = 0, gpus: int = 0) -> Dict[str, Any]:
    if provider == "aws":
        disks = [_disk("aws", boot_gb, False)] + ([_disk("aws", data_gb, True)] if data_gb else [])
        return {"InstanceType": instance, "BlockDeviceMappings": disks}
    if provider == "azure":
        p = {"vmSize": instance, "osDiskSizeGB": boot_gb}
        if data_gb:
            p["dataDisks"] = [{"lun": 0, "diskName": "datadisk1", "storageAccountType": "Premium_LRS",
                               "diskSizeGB": data_gb}]
        return {"azure_arm_parameters": p}
    if provider == "gcp":
        if isinstance(instance, tuple):
            machine, acc, n = instance
            extra = {"guestAccelerators": [{"acceleratorType": acc, "acceleratorCount": n}],
                     "scheduling": [{"onHostMaintenance": "TERMINATE"}]}
        else:
            machine, extra = instance, {}
        disks = [{"boot": True, "autoDelete": True, "type": "PERSISTENT",
                  "initializeParams": {"diskSizeGb": boot_gb}}]
        if data_gb:
            disks.append({"autoDelete": True, "type": "PERSISTENT",
                          "initializeParams": {"diskSizeGb": data_gb, "diskType": "pd-ssd"}})
        return dict({"machineType": machine, "disks": disks}, **extra)
    if provider == "aliyun":
        c = {"InstanceType": instance, "SystemDisk": {"Category": "cloud_essd", "Size": boot_gb}}
        if data_gb:
            c["DataDisk"] = [{"Category": "cloud_essd", "Size": data_gb, "DeleteWithInstance": True}]
        return c
    if provider == "huaweicloud":
        c = {"flavor": instance, "root_volume": {"volumetype": "SSD", "size": boot_gb}}
        if data_gb:
            c["data_volumes"] = [{"volumetype": "SSD", "size": data_gb}]
        return c
    raise KeyError(provider)


def _k8s(size: str, highmem: bool, cloud: Optional[str]) -> Dict[str, Any]:
    head_cpu, worker_cpu, data_gb = SIZES[size]
    per_cpu = 8 if highmem else 4
    sc = {"aws": "gp2", "azure": "managed-premium", "gcp": "standard-rwo"}.get(cloud or "", "standard")

    def pod(cpu, disk):
        # leave one vCPU and ~3 GiB per node for the kubelet / daemonsets
        return {"resources": {"cpu": max(1, cpu - 1), "memory": f"{max(2, cpu * per_cpu - 3)}Gi"},
                "dataDisks": [{"name": "data-disk-1", "storageClass": sc, "diskSize": f"{disk}Gi"}]}
    out = {"provider": {"type": "kubernetes"},
           "available_node_types": {"head.default": {"node_config": pod(head_cpu, 100)},
                                    "worker.default": {"node_config": pod(worker_cpu, data_gb)}}}
    if cloud:
        out["provider"]["cloud_provider"] = {"type": cloud}
    return out


def _size_parts(name: str) -> Tuple[str, bool]:
    highmem = name.endswith("-highmem")
    return (name[: -len("-highmem")] if highmem else name), highmem


def synthesize(name: str) -> Optional[Dict[str, Any]]:
    """The template called ``name`` (e.g. ``aws/standard``, ``gcp/gpu/t4/standard``,
    ``kubernetes/eks/small-highmem``, ``azure/latest/large``), or None if unknown."""
    parts = [p for p in name.replace(".yaml", "").split("/") if p]
    if not parts or parts[0] not in PROVIDERS:
        return None
    provider = parts[0]
    if provider == "kubernetes":
        cloud = None
        if len(parts) == 3 and parts[1] in K8S_CLOUDS:
            cloud, parts = K8S_CLOUDS[parts[1]], [parts[0], parts[2]]
        if len(parts) != 2:
            return None
        size, highmem = _size_parts(parts[1])
        return _k8s(size, highmem, cloud) if size in SIZES else None
    if len(parts) >= 2 and parts[1] == "gpu":
        return _gpu_template(provider, parts[2:])
    latest = len(parts) == 3 and parts[1] == "latest"
    if len(parts) != 2 and not latest:
        return None
    size, highmem = _size_parts(parts[-1])
    if size not in SIZES or provider not in _GENERAL:
        return None
    table = (_HIGHMEM if highmem else _GENERAL)[provider][1 if latest else 0]
    head_cpu, worker_cpu, data_gb = SIZES[size]
    return {"provider": {"type": provider},
            "available_node_types": {
                "head.default": {"node_config": _node_config(provider, table[head_cpu], 100)},
                "worker.default": {"node_config": _node_config(provider, table[worker_cpu], 100, data_gb)}}}


def _gpu_template(provider: str, rest: List[str]) -> Optional[Dict[str, Any]]:
    fams = _GPU.get(provider, {})
    general = _GENERAL.get(provider, ({},))[0]
    if len(rest) == 1 and rest[0].startswith("base"):
        # gpu/base[-N]: a head sized for driving N GPU workers
        n = int(rest[0].split("-")[1]) if "-" in rest[0] else 1
        head = general[16 if n <= 2 else 32]
        return {"provider": {"type": provider},
                "available_node_types": {"head.default": {"node_config": _node_config(provider, head, 256)}}}
    if len(rest) != 2 or rest[0] not in fams or rest[1] not in fams[rest[0]]:
        return None
    instance, gpus = fams[rest[0]][rest[1]]
    return {"provider": {"type": provider},
            "available_node_types": {
                "head.default": {"node_config": _node_config(provider, general[8 if gpus <= 2 else 16], 256)},
                "worker.default": {"node_config": _node_config(provider, instance, 256),
                                   "resources": {"GPU": gpus}}}}


def available() -> List[str]:
    """Every template name :func:`synthesize` knows."""
    out = []
    for p in PROVIDERS:
        sizes = [s + h for s in SIZES for h in ("", "-highmem")]
        if p == "kubernetes":
            out += [f"{p}/{s}" for s in sizes] + [f"{p}/{c}/{s}" for c in K8S_CLOUDS for s in sizes]
            continue
        out += [f"{p}/{s}" for s in sizes] + [f"{p}/latest/{s}" for s in sizes]
        for fam, tab in _GPU.get(p, {}).items():
            out += [f"{p}/gpu/{fam}/{s}" for s in tab]
        if p in _GPU:
            out += [f"{p}/gpu/base", f"{p}/gpu/base-2", f"{p}/gpu/base-4", f"{p}/gpu/base-8"]
    return out
