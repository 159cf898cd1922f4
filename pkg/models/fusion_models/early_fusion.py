from multimodal_alzheimer_amd.classifiers import PET_MRI_EF  # noqa: F401
from multimodal_alzheimer_amd.classifiers import Random_Benchmark_All_CN_EF as Random_Benchmark_All_CN  # noqa: F401,E501
