"""zoo.feature — FeatureSet (memory tiers, sharding), preprocessing, image/text pipelines."""
