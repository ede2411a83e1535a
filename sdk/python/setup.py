"""kubeflow-pytorchjob SDK for the MI355X-native operator."""
import setuptools

setuptools.setup(
    name="kubeflow-pytorchjob-amd",
    version="0.1.0",
    author="pytorch-operator-amd authors",
    description="PyTorchJob Python SDK (MI355X-native operator)",
    packages=["kubeflow", "kubeflow.pytorchjob", "kubeflow.pytorchjob.api", "kubeflow.pytorchjob.constants",
              "kubeflow.pytorchjob.models", "kubeflow.pytorchjob.utils"],
    python_requires=">=3.8",
    install_requires=["pyyaml"],  # + pytorch_operator_amd (cluster.rest transport)
)
