from multimodal_alzheimer_amd.classifiers import Small_PET_CNN, Random_Benchmark_All_CN  # noqa: F401
