from multimodal_alzheimer_amd.classifiers import PET_MRI_FMF  # noqa: F401
from multimodal_alzheimer_amd.classifiers import Random_Benchmark_All_CN_FMF as Random_Benchmark_All_CN  # noqa: F401,E501
