"""Spark runtime package: cluster API (``SparkCluster``) over the catalog runtime."""
