"""Drop-in for Density_aware_Chamfer_Distance/utils_v2/metrics/CD (chamfer3D + model_utils + fscore)."""
