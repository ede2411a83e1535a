"""kubeflow-pytorchjob: Python SDK for PyTorchJobs (MI355X-native operator).

Same distribution name and public API as the reference SDK (sdk/python/setup.py:26-61 of
jiaqianjing/pytorch-operator, ``kubeflow-pytorchjob`` 0.1.4); standalone: the transport is
the package's own stdlib ``rest`` module, so the only dependency is PyYAML (kubeconfig).
"""
import setuptools

setuptools.setup(
    name="kubeflow-pytorchjob",
    version="0.1.4",
    author="pytorch-operator-amd authors",
    description="Kubeflow PyTorchJob Python SDK (MI355X-native operator)",
    long_description=open(__file__.replace("setup.py", "README.md")).read(),
    long_description_content_type="text/markdown",
    packages=["kubeflow", "kubeflow.pytorchjob", "kubeflow.pytorchjob.api", "kubeflow.pytorchjob.constants",
              "kubeflow.pytorchjob.models", "kubeflow.pytorchjob.utils"],
    python_requires=">=3.8",
    install_requires=["pyyaml"],
    classifiers=["Programming Language :: Python :: 3", "License :: OSI Approved :: Apache Software License"],
)
