"""Drop-in alias: `import distilp` resolves to the MI355X-native distilp_amd package.

Code written against the reference (`from distilp.solver import halda_solve`,
`from distilp.common import DeviceProfile, ModelProfile`) runs unchanged.
"""

__version__ = "0.1.2"
