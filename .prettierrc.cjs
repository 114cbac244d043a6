module.exports = require('@headlamp-k8s/eslint-config/prettier-config');
