__path__ = __import__("pkgutil").extend_path(__path__, __name__)  # namespace package
